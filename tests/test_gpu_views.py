"""GPU: several row views in one call (per-island minibatches, src/SingleIteration.jl:40, 77).

`sr_eval_loss_batch_views` / `sr_eval_grad_batch_views` score tree t on the rows of its view in ONE
launch (tree groups view-pure: the interpreter's segments).  Each tree's loss, flags and gradient must
be bit-identical to `sr_eval_loss_batch` / `sr_eval_grad_batch` over its view alone (the same kernels
over the same rows), with BIG trees (the exact pass runs per view), weights, and views of a length that
is not a multiple of the row tile.  And a batching search scored on the device equals the same search
scored by the oracle.
"""
import numpy as np
import pytest

from sr_amd import (Dataset, Options, SubDataset, eval_grad_batch, eval_grad_batch_views, eval_loss_batch,
                    eval_loss_batch_views, flatten_trees, gen_random_population, parse_expression)

pytestmark = pytest.mark.gpu


def _setup(dtype, weighted, n=20000, n_views=7, view_len=1500, seed=3):
    rng = np.random.default_rng(seed)
    X = rng.standard_normal((5, n)).astype(dtype)
    X[2, ::97] = dtype(3e35 if dtype == np.float32 else 3e300)  # BIG trees over x3
    y = (2 * np.cos(X[3]) + X[0] ** 2 - 2).astype(dtype)
    w = (0.5 + rng.random(n)).astype(dtype) if weighted else None
    opts = Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp", "log"])
    trees = gen_random_population(900, opts, 5, max_size=25, dtype=dtype, seed=seed)
    trees += [parse_expression(e, opts) for e in ("x3 * 1.5", "x3 + x1", "(x3 * 0.5) - x2")]
    tb = flatten_trees(trees, dtype)
    views = rng.integers(0, n, (n_views, view_len))
    tree_view = rng.integers(0, n_views, tb.n_trees)
    return Dataset(X, y, weights=w), opts, tb, views, tree_view


@pytest.mark.parametrize("dtype,weighted", [(np.float32, False), (np.float32, True), (np.float64, True)])
def test_loss_views_equal_per_view_calls(dtype, weighted):
    ds, opts, tb, views, tree_view = _setup(dtype, weighted)
    loss, comp = eval_loss_batch_views(tb, ds, opts, tree_view, views)
    n_big = 0
    for v in range(views.shape[0]):
        sel = np.nonzero(tree_view == v)[0]
        lv, cv = eval_loss_batch(tb.take(sel), SubDataset(ds, views[v]), opts)
        assert np.array_equal(comp[sel], cv), v
        assert np.array_equal(loss[sel].view(np.uint8), lv.view(np.uint8)), v
        n_big += int(np.sum(cv[-3:])) if v == tree_view[-1] else 0
    assert 0.1 < comp.mean() < 0.95


def test_grad_views_equal_per_view_calls():
    ds, opts, tb, views, tree_view = _setup(np.float64, True, n=8000, view_len=700, seed=5)
    loss, g, comp = eval_grad_batch_views(tb, ds, opts, tree_view, views)
    co = tb.constant_offsets()
    for v in range(views.shape[0]):
        sel = np.nonzero(tree_view == v)[0]
        lv, gv, cv = eval_grad_batch(tb.take(sel), SubDataset(ds, views[v]), opts)
        assert np.array_equal(comp[sel], cv)
        assert np.array_equal(loss[sel].view(np.uint8), lv.view(np.uint8))
        sub_co = tb.take(sel).constant_offsets()
        for j, t in enumerate(sel):
            assert np.array_equal(g[co[t]:co[t + 1]].view(np.uint8), gv[sub_co[j]:sub_co[j + 1]].view(np.uint8)), (v, t)


@pytest.mark.parametrize("optimize", [False, True])
def test_batching_search_device_equals_oracle_scored(optimize):
    """A batching search (one minibatch per island and iteration, one more for the optimiser): scored on
    the device (every island's trees in one launch per round) and by the oracle (one call per view)
    -> identical populations when the constant optimiser is off; with it on (BFGS is chaotic in the
    last bits) every stored loss equals the oracle's re-evaluation on the full data."""
    from oracle import Oracle
    from sr_amd import equation_search, string_tree

    rng = np.random.default_rng(11)
    X = rng.uniform(0.5, 2.0, (5, 20000)).astype(np.float32)
    y = (X[0] * X[1] * X[2] / (X[3] * X[4] ** 2 + 1)).astype(np.float32)
    opts = Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp", "log"], populations=5,
                   population_size=20, ncycles_per_iteration=10, maxsize=20, batching=True, batch_size=700,
                   should_optimize_constants=optimize, optimizer_probability=0.3)
    orc = Oracle.from_options(opts)

    def oracle_loss(tb, rows):
        Xv, yv = (X, y) if rows is None else (X[:, rows], y[rows])
        losses, comp = orc.eval_loss_batch(tb, Xv, yv, accum="ref", n_threads=8)  # (the reference's fold)
        return np.where(comp, losses, np.inf)

    dev = equation_search(X, y, niterations=2, options=opts, seed=5, scoring_lanes=1)
    if not optimize:
        ref = equation_search(X, y, niterations=2, options=opts, seed=5, _loss_fn=oracle_loss)
        assert [[string_tree(m.tree, opts.operators) for m in p] for p in dev.populations] == \
               [[string_tree(m.tree, opts.operators) for m in p] for p in ref.populations]
        assert dev.device_calls == ref.device_calls
    members = [m for p in dev.populations for m in p]
    ol, oc = orc.eval_loss_batch(flatten_trees([m.tree for m in members], np.float32), X, y, accum="f64", n_threads=8)
    stored = np.array([m.loss for m in members], dtype=np.float64)
    assert np.array_equal(np.isfinite(stored), oc)
    fin = np.isfinite(stored)
    np.testing.assert_allclose(stored[fin], ol[fin], rtol=1e-4)  # finalize_costs: the full data
