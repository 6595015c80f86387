"""CPU: the search restatement's selection / bookkeeping rules (oracle/search_oracle.py).

The native engine (csrc/sr_search.cpp) is pinned to this restatement trajectory for trajectory in
tests/test_search_engine.py; the rules themselves are pinned here against the reference:
tournament selection statistics (test/unit/evolution-core/test_prob_pick_first.jl:1-53), ranking
with NaN / Inf costs (argmin_fast / bottomk_fast, src/Utils.jl:96-147), adjusted costs computed in
L (src/Population.jl:124-139), the Pareto frontier (src/HallOfFame.jl:96-124), the
adaptive-parsimony window (src/AdaptiveParsimony.jl:55-93), loss_to_cost (src/LossFunctions.jl:
169-190), and that every mutation (src/MutationFunctions.jl) yields a well-formed tree.
"""
import numpy as np
import pytest

import bytecode_vm as vm
import search_oracle as so_mod
from sr_amd import Node, Options, SearchOptions, flatten_trees, parse_expression

OPTS = dict(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "sin"])


def _oracle(opts, so=None, T=np.float64, seed=0):
    o = so_mod.SearchOracle(opts, so or SearchOptions(), 3, 10, T, seed, lambda trees, rows=None: np.zeros(len(trees)))
    o.snap = [[1.0 / opts.maxsize] * opts.maxsize for _ in range(opts.populations)]
    o.baseline, o.use_baseline = T(1), True
    return o


def _member(tree, cost, loss=1.0):
    return so_mod.Member(tree, cost, loss, tree.count_nodes(), 0, 0)


@pytest.mark.parametrize("reverse", [False, True])
def test_tournament_selection_prefers_low_cost(reverse):
    n = 10
    opts = Options(**OPTS, tournament_selection_p=0.999, tournament_selection_n=n, populations=1)
    o = _oracle(opts)
    trees = [parse_expression("x1", opts) for _ in range(n)]
    o.pops = [[_member(trees[i], (1 - i / (n - 1)) if reverse else i / (n - 1)) for i in range(n)]]
    picks = [o.best_of_sample(0).cost for _ in range(100)]
    assert np.mean(picks) < 0.1


def test_tournament_ranking_skips_nan_and_inf():
    opts = Options(**OPTS, tournament_selection_p=1.0, tournament_selection_n=4, populations=1)
    o = _oracle(opts, SearchOptions(use_frequency_in_tournament=False))
    t = parse_expression("x1", opts)
    o.pops = [[_member(t, np.nan), _member(t, np.inf), _member(t, 0.5), _member(t, 0.2)]]
    for _ in range(10):
        assert o.best_of_sample(0).cost == 0.2
    # no finite cost at all: argmin_fast keeps its initial index, the first sampled member
    o.pops = [[_member(t, np.nan), _member(t, np.inf)]]
    o.o.tournament_selection_n = 2
    for _ in range(5):
        assert not np.isfinite(o.best_of_sample(0).cost)


def test_tournament_adjusted_costs_in_loss_type():
    """adjusted_costs::Vector{L} = cost * exp(L(scaling) * L(freq)) in L (Float32 for Float32 data):
    two members whose Float32 adjusted costs tie (but whose float64 ones do not) keep the first
    sampled member (argmin_fast: strict <)."""
    c = np.float32(1.0320923328399658)
    f1, f2 = 0.11347446513971259, 0.11347445643963802
    assert float(c) * np.exp(20.0 * f2) < float(c) * np.exp(20.0 * f1)  # float64 would pick m2
    opts = Options(**OPTS, tournament_selection_n=2, tournament_selection_p=1.0, populations=1, maxsize=30)
    o = _oracle(opts, SearchOptions(adaptive_parsimony_scaling=20.0), T=np.float32)
    m1 = _member(parse_expression("x1 + x2", opts), c)
    m2 = _member(parse_expression("x1 + cos(x2)", opts), c)
    assert (m1.complexity, m2.complexity) == (3, 4)
    freqs = [0.0] * 30
    freqs[2], freqs[3] = f1, f2
    o.snap = [freqs]
    for seed in range(6):
        o.rngs = [so_mod.Rng(seed, 0)]
        o.pops = [[m1, m2]]
        first = so_mod.Rng(seed, 0).below(2)  # the partial Fisher-Yates' first pick
        won = o.best_of_sample(0)
        assert won.complexity == [m1, m2][first].complexity, seed


def test_pareto_frontier_and_hall_of_fame():
    opts = Options(**OPTS, populations=1)
    o = _oracle(opts)
    o.hof = [None] * opts.maxsize
    exprs = ["x1", "cos(x1)", "x1 * x2", "cos(x1 * x2)", "x1 * x2 + 1.0"]
    losses = [4.0, 5.0, 2.0, 3.0, 1.0]
    for e, l in zip(exprs, losses):
        o.hof_update(_member(parse_expression(e, opts), l, l))
    # sizes 1 (4.0), 2 (5.0: not below size 1), 3 (2.0), 4 (3.0: not below size 3), 5 (1.0)
    assert [m.complexity for m in o.pareto()] == [1, 3, 5]
    o.hof_update(_member(parse_expression("x2", opts), 0.5, 0.5))
    assert [m.complexity for m in o.pareto()] == [1]


def test_running_statistics_window():
    opts = Options(**OPTS, populations=1, maxsize=10)
    o = _oracle(opts)
    o.freq = [1.0] * 10
    for size in [3] * 200_000 + [5] * 50_000:
        o.freq[size - 1] += 1.0
    o.move_window()
    assert abs(sum(o.freq) - 100_000) < 1e-3 and min(o.freq) >= 1
    nf = o.normalized()
    assert abs(sum(nf) - 1) < 1e-12 and nf[2] > nf[4] >= nf[0]


def test_every_mutation_gives_valid_programs():
    opts = Options(**OPTS, maxsize=20)
    sp = so_mod.Spec(opts, SearchOptions(), 3, np.float32)
    rng = so_mod.Rng(5, 0)
    base = [so_mod.gen_random_tree(3, sp, rng) for _ in range(40)]
    trees = []
    for choice in so_mod.MUTATIONS:
        if choice in ("simplify", "do_nothing", "optimize"):
            continue
        for t in base:
            trees.append(so_mod.mutate(t.copy(), choice, sp, 0.5, opts.maxsize, rng))
    for a, b in zip(base[::2], base[1::2]):
        trees.extend(so_mod.crossover(a, b, rng))
        trees.append(so_mod.simplify(a.copy(), sp))
    tb = flatten_trees(trees, np.float32)
    vm.compile_info(opts, tb, 64, 3, np.float32)  # the device compiler accepts every produced tree
    assert all(t.count_nodes() >= 1 for t in trees)


def test_simplify_folds_constants_and_combines():
    opts = Options(binary_operators=["+", "-", "*"], unary_operators=["cos"])
    sp = so_mod.Spec(opts, SearchOptions(), 2, np.float64)
    t = so_mod.simplify(parse_expression("(x1 + 2.0) + 3.0", opts), sp)
    assert t.count_nodes() == 3 and sorted([n.val for n in t.preorder() if n.constant]) == [5.0]
    t = so_mod.simplify(parse_expression("cos(0.0) * x2", opts), sp)
    assert [n.val for n in t.preorder() if n.constant] == [1.0]
    t = so_mod.simplify(parse_expression("(x1 - 1.5) - 2.0", opts), sp)
    assert t.count_nodes() == 3 and [n.val for n in t.preorder() if n.constant] == [3.5]


def test_costs_match_loss_to_cost():
    """The search's cost (loss_to_cost in L with the Float32 parsimony product) == sr_amd.loss_to_cost."""
    from sr_amd import loss_to_cost

    opts = Options(binary_operators=["+", "*"], unary_operators=["cos"], parsimony=0.0032, populations=1)
    for dt in (np.float32, np.float64):
        o = _oracle(opts, T=dt)
        for use, base in ((True, 3.7), (True, 0.001), (False, 5.0)):
            o.use_baseline, o.baseline = use, dt(base)
            for loss, size in ((0.0, 1), (1.5, 3), (1e-7, 30), (np.inf, 7), (123.25, 12)):
                want = loss_to_cost(dt(loss), use, dt(base), Node(val=dt(0)), opts, size)
                assert o.cost_of(dt(loss), size) == want
