"""CPU: the native search engine (csrc/sr_search.cpp through the C ABI) equals its independent
Python restatement (oracle/search_oracle.py) trajectory for trajectory.

Both run the same seeded search with the same scorer (the C oracle, through the engine's CPU
callback hook): every population member (tree, cost, birth, ref, parent) and the Pareto front must
be identical after several iterations, across Float32 / Float64, crossover-heavy runs, kept
mutation failures, maxsize warm-up and with or without simplification.  Property checks on the
engine itself follow (constraints, determinism, the island exchange round trip, option validation).
"""
import ctypes

import numpy as np
import pytest

from oracle import Oracle
from search_oracle import SearchOracle
from sr_amd import Options, SearchOptions, _lib, flatten_trees
from sr_amd.search import NativeSearch, equation_search


def _data(dtype, n=60, seed=0):
    rng = np.random.default_rng(seed)
    X = rng.standard_normal((2, n)).astype(dtype)
    y = (2 * np.cos(X[1]) + X[0] ** 2 - 2).astype(dtype)
    return X, y


def _loss_fn(opts, X, y):
    orc = Oracle.from_options(opts)

    def lf(tb, rows):
        Xv, yv = (X, y) if rows is None else (X[:, rows], y[rows])
        losses, comp = orc.eval_loss_batch(tb, Xv, yv, accum="ref")
        return np.where(comp, losses, np.inf)

    return lf


def _restated_loss(lf, dtype):
    """The restatement's loss_fn(trees, rows): rows None (full data) or one row array per tree (its
    island's minibatch)."""
    def f(trees, rows):
        if rows is None:
            return lf(flatten_trees(trees, dtype), None)
        out = np.empty(len(trees))
        groups = {}
        for k, r in enumerate(rows):
            groups.setdefault(id(r), (r, []))[1].append(k)
        for r, ks in groups.values():
            out[ks] = lf(flatten_trees([trees[k] for k in ks], dtype), r)
        return out
    return f


def _key(t, dtype):
    tb = flatten_trees([t], dtype)
    return tuple(tb.degree), tuple(tb.op), tuple(tb.feature), tuple(float(v) for v in tb.val)


CASES = [
    ("f64", np.float64, 1, {}, {}),
    ("f32", np.float32, 2, {}, {}),
    ("crossover_keep_failures", np.float64, 3, dict(skip_mutation_failures=False, crossover_probability=0.3), {}),
    ("warmup_no_simplify_f32", np.float32, 4, dict(warmup_maxsize_by=0.5, should_simplify=False), {}),
    ("no_annealing_no_frequency", np.float64, 5, dict(annealing=False, use_frequency=False,
                                                      use_frequency_in_tournament=False), {}),
    ("tournament_p1_parsimony", np.float32, 6, {}, dict(tournament_selection_p=1.0, parsimony=0.01)),
    ("heavy_migration", np.float64, 7, dict(fraction_replaced=0.2, fraction_replaced_hof=0.3, topn=4), {}),
    # per-island minibatches (src/SingleIteration.jl:40): each island's children on its own rows
    ("batching_f32", np.float32, 8, {}, dict(batching=True, batch_size=17)),
    ("batching_f64_crossover", np.float64, 9, dict(crossover_probability=0.3), dict(batching=True, batch_size=23)),
]


@pytest.mark.parametrize("name,dtype,seed,sokw,okw", CASES, ids=[c[0] for c in CASES])
def test_engine_equals_restatement(name, dtype, seed, sokw, okw):
    so = SearchOptions(**sokw)
    opts = Options(binary_operators=["+", "*", "/", "-"], unary_operators=["cos", "exp"], populations=3,
                   population_size=12, ncycles_per_iteration=15, maxsize=15, should_optimize_constants=False, **okw)
    X, y = _data(dtype)
    lf = _loss_fn(opts, X, y)
    res = equation_search(X, y, niterations=3, options=opts, seed=seed, search_options=so, _loss_fn=lf)
    ref = SearchOracle(opts, so, 2, X.shape[1], dtype, seed, _restated_loss(lf, dtype)).run(3)
    for i, (pa, pb) in enumerate(zip(res.populations, ref.pops)):
        for k, (a, b) in enumerate(zip(pa, pb)):
            assert (_key(a.tree, dtype), float(a.cost), a.birth, a.ref, a.parent) == \
                   (_key(b.tree, dtype), float(b.cost), b.birth, b.ref, b.parent), (name, i, k)
    assert [(_key(m.tree, dtype), float(m.loss)) for m in res.pareto_frontier] == \
           [(_key(m.tree, dtype), float(m.loss)) for m in ref.pareto()]
    assert res.device_calls == ref.calls


def test_engine_members_respect_constraints_and_are_deterministic():
    opts = Options(binary_operators=["+", "*", "-"], unary_operators=["cos"], populations=4, population_size=15,
                   ncycles_per_iteration=20, maxsize=12, maxdepth=6, should_optimize_constants=False)
    X, y = _data(np.float64, n=40, seed=2)
    lf = _loss_fn(opts, X, y)
    runs = [equation_search(X, y, niterations=3, options=opts, seed=11, _loss_fn=lf) for _ in range(2)]
    for res in runs:
        for pop in res.populations:
            assert len(pop) == opts.population_size
            for m in pop:
                assert m.tree.count_nodes() <= opts.maxsize and m.tree.count_depth() <= opts.maxdepth
        for s, (m, e) in enumerate(zip(res.hall_of_fame.members, res.hall_of_fame.exists)):
            if e:
                assert m.complexity == s + 1 == m.tree.count_nodes()
        losses = [m.loss for m in res.pareto_frontier]
        assert all(a > b for a, b in zip(losses, losses[1:]))  # each front member beats every simpler one
    key = [[(_key(m.tree, np.float64), m.birth) for m in p] for p in runs[0].populations]
    assert key == [[(_key(m.tree, np.float64), m.birth) for m in p] for p in runs[1].populations]
    assert runs[0].device_calls == 1 + 1 + 3 * 20 * 1  # baseline, initial populations, one per round


def test_island_exchange_round_trip():
    """A rank's export imported into another engine reproduces its islands exactly."""
    opts = Options(binary_operators=["+", "*"], unary_operators=["cos"], populations=4, population_size=10,
                   ncycles_per_iteration=5, maxsize=10, should_optimize_constants=False)
    X, y = _data(np.float32, n=30, seed=4)
    lf = _loss_fn(opts, X, y)
    ds = type("D", (), {"dtype": np.dtype(np.float32), "nfeatures": 2, "n": 30})()
    a = NativeSearch(ds, opts, SearchOptions(), seed=3, rank=0, world=2)
    b = NativeSearch(ds, opts, SearchOptions(), seed=3, rank=1, world=2)
    for e in (a, b):
        e.use_callbacks(lf)
        e.start(2)
    a.iterate()
    b.import_(a.export())  # rank 1 now holds rank 0's islands 0 and 2
    for i in (0, 2):
        ma, mb = a.members(i), b.members(i)
        assert [(_key(m.tree, np.float32), float(m.cost), m.birth, m.ref) for m in ma] == \
               [(_key(m.tree, np.float32), float(m.cost), m.birth, m.ref) for m in mb]
    with pytest.raises(_lib.SRError):
        b.import_(a.export()[:-3])  # truncated buffers are refused


def test_engine_rejects_bad_arguments():
    opts = Options(binary_operators=["+"], unary_operators=[], populations=2, population_size=5, maxsize=5)
    o = _lib.SrSearchOptions()
    h = ctypes.c_void_p()
    un = (ctypes.c_char_p * 1)()
    bi = (ctypes.c_char_p * 1)(b"+")
    assert _lib.lib.sr_search_create(0, 2, 10, 0, un, 1, bi, ctypes.byref(o), 1, 0, 1, ctypes.byref(h)) \
        == _lib.SR_ERR_INVALID_ARG  # all-zero options
    bad = (ctypes.c_char_p * 1)(b"no_such_op")
    from sr_amd.search import search_options_struct

    so = search_options_struct(opts, SearchOptions())
    assert _lib.lib.sr_search_create(0, 2, 10, 0, un, 1, bad, ctypes.byref(so), 1, 0, 1, ctypes.byref(h)) \
        == _lib.SR_ERR_UNSUPPORTED_OP
    assert _lib.lib.sr_search_create(0, 2, 10, 0, un, 1, bi, ctypes.byref(so), 1, 2, 2, ctypes.byref(h)) \
        == _lib.SR_ERR_INVALID_ARG  # rank outside the world
    assert _lib.lib.sr_search_create(0, 2, 10, 0, un, 1, bi, ctypes.byref(so), 1, 0, 1, ctypes.byref(h)) == 0
    assert _lib.lib.sr_search_iterate(h) == _lib.SR_ERR_INVALID_ARG  # not started
    assert _lib.lib.sr_search_start(h, 1) == _lib.SR_ERR_INVALID_ARG  # no scorer
    assert _lib.lib.sr_search_free(h) == 0
