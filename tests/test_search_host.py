"""CPU: host-side search logic of sr_amd.search (no device calls).

Mirrors the reference's evolution-core unit tests: tournament selection statistics
(test/unit/evolution-core/test_prob_pick_first.jl:1-53), the Pareto frontier
(src/HallOfFame.jl:96-124), the adaptive-parsimony window (src/AdaptiveParsimony.jl:55-93) and
that every mutation (src/MutationFunctions.jl) yields a well-formed tree within the constraints.
"""
import numpy as np
import pytest

import bytecode_vm as vm
from sr_amd import Options, flatten_trees, gen_random_population
from sr_amd.search import (MUTATIONS, HallOfFame, PopMember, RunningSearchStatistics, SearchOptions, best_of_sample,
                           check_constraints, condition_mutation_weights, crossover_trees, mutate,
                           random_population_trees, replace_oldest, tournament_selection_weights)

OPTS = dict(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "sin"])


def _member(tree, cost, loss=1.0):
    return PopMember(tree, cost, loss, tree.count_nodes())


@pytest.mark.parametrize("reverse", [False, True])
def test_tournament_selection_prefers_low_cost(reverse):
    n = 10
    opts = Options(**OPTS, tournament_selection_p=0.999, tournament_selection_n=n)
    so = SearchOptions()
    rng = np.random.default_rng(0)
    trees = gen_random_population(n, opts, 2, seed=3)
    members = []
    for i in range(n):
        cost = np.float32(i) / (n - 1)
        members.append(_member(trees[i], 1 - cost if reverse else cost))
    stats = RunningSearchStatistics(opts.maxsize)
    w = tournament_selection_weights(opts)
    picks = [best_of_sample(members, stats, opts, so, rng, w).cost for _ in range(100)]
    assert np.mean(picks) < 0.1


def test_tournament_ranking_skips_nan_and_inf():
    opts = Options(**OPTS, tournament_selection_p=1.0, tournament_selection_n=4)
    so = SearchOptions(use_frequency_in_tournament=False)
    t = gen_random_population(4, opts, 2, seed=1)
    members = [_member(t[0], np.nan), _member(t[1], np.inf), _member(t[2], 0.5), _member(t[3], 0.2)]
    rng = np.random.default_rng(1)
    stats = RunningSearchStatistics(opts.maxsize)
    for _ in range(10):
        assert best_of_sample(members, stats, opts, so, rng, tournament_selection_weights(opts)).cost == 0.2


def test_pareto_frontier_and_hall_of_fame():
    opts = Options(**OPTS)
    hof = HallOfFame(opts.maxsize)
    trees = {s: gen_random_population(1, opts, 2, max_size=1, seed=s)[0] for s in range(3)}
    from sr_amd import parse_expression

    exprs = ["x1", "cos(x1)", "x1 * x2", "cos(x1 * x2)", "x1 * x2 + 1.0"]
    losses = [4.0, 5.0, 2.0, 3.0, 1.0]
    members = [_member(parse_expression(e, opts), l, l) for e, l in zip(exprs, losses)]
    hof.update(members, opts, opts.maxsize)
    front = hof.pareto_frontier()
    # sizes 1 (4.0), 2 (5.0: not better than size 1), 3 (2.0), 4 (3.0: worse than size 3), 5 (1.0)
    assert [m.complexity for m in front] == [1, 3, 5]
    # a better member of an existing size replaces it
    hof.update([_member(parse_expression("x2", opts), 0.5, 0.5)], opts, opts.maxsize)
    assert [m.complexity for m in hof.pareto_frontier()] == [1]
    del trees


def test_running_statistics_window():
    s = RunningSearchStatistics(10, window_size=100)
    for size in [3] * 200 + [5] * 50:
        s.update_frequencies(size)
    s.move_window()
    assert abs(s.frequencies.sum() - 100) < 1e-6 and np.all(s.frequencies >= 1)
    s.normalize_frequencies()
    assert abs(s.normalized_frequencies.sum() - 1) < 1e-12
    assert s.normalized_frequencies[2] > s.normalized_frequencies[4] >= s.normalized_frequencies[0]


def test_every_mutation_gives_valid_programs():
    opts = Options(**OPTS, maxsize=20)
    so = SearchOptions()
    rng = np.random.default_rng(5)
    base = random_population_trees(40, opts, 3, np.float32, rng)
    trees = []
    for choice in MUTATIONS:
        for t in base:
            m = mutate(t.copy(), choice, opts, so, 0.5, opts.maxsize, 3, np.float32, rng)
            trees.append(m)
    for a, b in zip(base[::2], base[1::2]):
        trees.extend(crossover_trees(a, b, rng))
    tb = flatten_trees(trees, np.float32)
    # the device compiler accepts every produced tree (no malformed pre-order arrays)
    vm.compile_info(opts, tb, 64, 3, np.float32)
    assert all(t.count_nodes() >= 1 for t in trees)


def test_condition_weights_and_constraints():
    from sr_amd import parse_expression

    opts = Options(**OPTS, maxsize=7, maxdepth=4)
    so = SearchOptions()
    leaf = _member(parse_expression("x1", opts), 1.0)
    w = condition_mutation_weights(so.mutation_weights, leaf, so, opts.maxsize, 3)
    assert w["mutate_operator"] == 0 and w["mutate_constant"] == 0 and w["delete_node"] == 0
    big = _member(parse_expression("cos(x1 * x2) + x3", opts), 1.0)
    w = condition_mutation_weights(so.mutation_weights, big, so, 6, 3)
    assert w["add_node"] == 0 and w["insert_node"] == 0  # complexity 6 >= curmaxsize
    assert check_constraints(big.tree, opts, 7) and not check_constraints(big.tree, opts, 5)
    deep = parse_expression("cos(cos(cos(cos(x1))))", opts)
    assert not check_constraints(deep, opts, 7)  # depth 5 > maxdepth 4


def test_replace_oldest():
    opts = Options(**OPTS)
    t = gen_random_population(3, opts, 2, seed=2)
    pop = [_member(x, 1.0) for x in t]
    oldest = pop[0]
    replace_oldest(pop, [_member(t[0].copy(), 0.0)])
    assert oldest not in pop and len(pop) == 3


def test_vectorised_costs_match_loss_to_cost():
    """search._costs (the batched loss_to_cost the search uses) == loss_to_cost tree by tree."""
    from sr_amd import Dataset, Node, Options, loss_to_cost
    from sr_amd.search import _costs

    opts = Options(binary_operators=["+", "*"], unary_operators=["cos"], parsimony=0.0032)
    for dt in (np.float32, np.float64):
        ds = Dataset(np.zeros((2, 10), dtype=dt), np.zeros(10, dtype=dt))
        for use, base in ((True, 3.7), (True, 0.001), (False, 5.0)):
            ds.use_baseline, ds.baseline_loss = use, dt(base)
            losses = np.array([0.0, 1.5, 1e-7, np.inf, 123.25], dtype=dt)
            sizes = np.array([1, 3, 30, 7, 12])
            got = _costs(losses, sizes, ds, opts)
            want = [float(loss_to_cost(losses[k], ds.use_baseline, ds.baseline_loss, Node(val=dt(0)), opts,
                                       int(sizes[k]))) for k in range(len(sizes))]
            assert got.tolist() == want


def test_tournament_adjusted_costs_in_loss_type():
    """src/Population.jl:124-139 computes adjusted_costs::Vector{L} = cost * exp(L(scaling) * L(freq))
    in L (Float32 for Float32 data).  Two members whose Float32 adjusted costs tie but whose float64
    ones do not: the tie keeps the first member of the sample (argmin_fast: strict <)."""
    from types import SimpleNamespace

    from sr_amd.search import best_of_sample

    c = np.float32(1.0320923328399658)
    f1, f2 = 0.11347446513971259, 0.11347445643963802  # L(f1) != L(f2); exp products tie in Float32
    m1 = SimpleNamespace(cost=c, complexity=3, name="m1")
    m2 = SimpleNamespace(cost=c, complexity=4, name="m2")
    freqs = np.zeros(30)
    freqs[2], freqs[3] = f1, f2
    stats = SimpleNamespace(normalized_frequencies=freqs)
    options = SimpleNamespace(tournament_selection_n=2, tournament_selection_p=1.0, maxsize=30)
    so = SimpleNamespace(use_frequency_in_tournament=True, adaptive_parsimony_scaling=20.0)
    assert float(c) * np.exp(20.0 * f2) < float(c) * np.exp(20.0 * f1)  # float64 would pick m2
    for seed in range(6):
        order = np.random.default_rng(seed).choice(2, size=2, replace=False)
        won = best_of_sample([m1, m2], stats, options, so, np.random.default_rng(seed), None)
        assert won is [m1, m2][order[0]], seed  # Float32 tie: the first sampled member wins
