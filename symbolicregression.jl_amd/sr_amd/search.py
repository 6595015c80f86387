"""``equation_search`` host loop with lock-step islands (§8(a) A9, A10).

Restates the reference's search around the device scoring path:
  * ``_main_search_loop!`` / ``_dispatch_s_r_cycle`` (src/SymbolicRegression.jl:967-1296):
    per iteration every island runs ``s_r_cycle``, then ``optimize_and_simplify_population``; the
    head updates the running search statistics, the hall of fame, the Pareto frontier and
    migrates members (``migrate!``, src/Migration.jl:15-37);
  * ``s_r_cycle`` (src/SingleIteration.jl:19-66): ``ncycles_per_iteration`` annealing
    temperatures LinRange(1, 0), one ``reg_evol_cycle`` each, best-seen per complexity;
  * ``reg_evol_cycle`` (src/RegularizedEvolution.jl:12-160): ceil(n / tournament_n) rounds of
    tournament selection (``best_of_sample``, src/Population.jl:84-134), mutation
    (``next_generation``, src/Mutate.jl:184-356) or crossover (``crossover_generation``, :661-733),
    replacing the oldest member;
  * mutation operators of src/MutationFunctions.jl and the weights of src/MutationWeights.jl /
    the v1 defaults (src/Options.jl:1161-1208).

MI355X-first change (the point of the exercise): the islands advance in LOCK-STEP.  At every
regularised-evolution round, each island does its host-side selection and mutation, and the
children of ALL islands are scored by ONE batched ``eval_cost`` launch; the per-island serial
semantics (each island's next round sees its own previous replacement) are kept.  Constant
optimisation at the end of an iteration runs batched over all islands' selected members
(``optimize_constants_batch``).  The islands of one iteration share one snapshot of the running
search statistics (the reference's serial scheduler hands each island the snapshot current at its
dispatch); random streams are per island (numpy PCG64), not Julia's, so trajectories are
reproducible run to run (``seed``) but not equal to a Julia run's.
"""
from __future__ import annotations

import math
import time
from dataclasses import dataclass, field

import numpy as np

from . import _lib

from .constant_optimization import optimize_constants_batch
from .dataset import Dataset, batch
from .loss import eval_cost_batch, eval_loss_batch, loss_to_cost, update_baseline_loss_
from .mutation import gen_random_tree_fixed_size, make_random_leaf
from .node import Node, flatten_trees

MUTATIONS = ("mutate_constant", "mutate_operator", "mutate_feature", "swap_operands", "rotate_tree", "add_node",
             "insert_node", "delete_node", "simplify", "randomize", "do_nothing", "optimize")

# v1 defaults (src/Options.jl:1174-1188); form/break_connection are 0 for plain Node trees
DEFAULT_MUTATION_WEIGHTS = dict(mutate_constant=0.0346, mutate_operator=0.293, mutate_feature=0.1,
                                swap_operands=0.198, rotate_tree=4.26, add_node=2.47, insert_node=0.0112,
                                delete_node=0.870, simplify=0.00209, randomize=0.000502, do_nothing=0.273,
                                optimize=0.0)


@dataclass
class SearchOptions:
    """Search knobs with the reference's v1 defaults (src/Options.jl:1161-1208)."""
    crossover_probability: float = 0.0259
    annealing: bool = True
    alpha: float = 3.17
    perturbation_factor: float = 0.129
    probability_negate_constant: float = 0.00743
    use_frequency: bool = True
    use_frequency_in_tournament: bool = True
    adaptive_parsimony_scaling: float = 1040.0
    fraction_replaced: float = 0.00036
    fraction_replaced_hof: float = 0.0614
    topn: int = 12
    migration: bool = True
    hof_migration: bool = True
    skip_mutation_failures: bool = True
    should_simplify: bool = False  # simplify_tree!/combine_operators live in DynamicExpressions
    warmup_maxsize_by: float = 0.0
    mutation_weights: dict = field(default_factory=lambda: dict(DEFAULT_MUTATION_WEIGHTS))


# ---------------------------------------------------------------------------------- members
class _Counter:
    def __init__(self):
        self.v = 0

    def __call__(self):
        self.v += 1
        return self.v


_next_ref = _Counter()
_next_birth = _Counter()


class PopMember:
    """src/PopMember.jl: tree, cost, loss, birth order, complexity, ref / parent."""
    __slots__ = ("tree", "cost", "loss", "birth", "complexity", "ref", "parent")

    def __init__(self, tree, cost, loss, complexity, parent=-1, birth=None):
        self.tree = tree
        self.cost = float(cost)
        self.loss = float(loss)
        self.complexity = int(complexity)
        self.birth = _next_birth() if birth is None else birth
        self.ref = _next_ref()
        self.parent = parent

    def copy(self):
        m = PopMember.__new__(PopMember)
        m.tree = self.tree.copy()
        m.cost, m.loss, m.birth, m.complexity, m.ref, m.parent = (self.cost, self.loss, self.birth, self.complexity,
                                                                    self.ref, self.parent)
        return m


class RunningSearchStatistics:
    """src/AdaptiveParsimony.jl:20-93."""

    def __init__(self, maxsize, window_size=100000):
        self.window_size = window_size
        self.frequencies = np.ones(maxsize)
        self.normalized_frequencies = self.frequencies / self.frequencies.sum()

    def update_frequencies(self, size):
        if 0 < size <= len(self.frequencies):
            self.frequencies[size - 1] += 1

    def move_window(self):
        f = self.frequencies
        diff = f.sum() - self.window_size
        loops = 0
        while diff > 0:
            idx = np.nonzero(f > 1)[0]
            if len(idx) == 0:
                break
            amount = min(diff / len(idx), f[idx].min() - 1)
            f[idx] -= amount
            total = amount * len(idx)
            diff -= total
            loops += 1
            if loops > 1000 or total < 1e-6:
                break

    def normalize_frequencies(self):
        self.normalized_frequencies = self.frequencies / self.frequencies.sum()

    def copy(self):
        s = RunningSearchStatistics.__new__(RunningSearchStatistics)
        s.window_size = self.window_size
        s.frequencies = self.frequencies.copy()
        s.normalized_frequencies = self.normalized_frequencies.copy()
        return s


def check_constraints(tree, options, maxsize, size=None):
    """check_constraints (src/CheckConstraints.jl:75-92): size and depth limits."""
    size = size if size is not None else tree.count_nodes()
    if size > maxsize:
        return False
    return size <= options.maxdepth or tree.count_depth() <= options.maxdepth  # depth <= node count


class HallOfFame:
    """Best member per complexity (src/HallOfFame.jl; update_hall_of_fame!, src/SearchUtils.jl:717-736)."""

    def __init__(self, maxsize):
        self.members = [None] * maxsize
        self.exists = [False] * maxsize

    def update(self, members, options, maxsize):
        for m in members:
            size = m.complexity
            if not (0 < size <= maxsize) or not check_constraints(m.tree, options, maxsize, size):
                continue
            cur = self.members[size - 1]
            if not self.exists[size - 1] or m.cost < cur.cost:
                self.members[size - 1] = m.copy()
                self.exists[size - 1] = True

    def pareto_frontier(self):
        """calculate_pareto_frontier (src/HallOfFame.jl:96-124): a member is kept when its loss is
        below that of every existing simpler member."""
        out = []
        for size in range(len(self.members)):
            if not self.exists[size]:
                continue
            m = self.members[size]
            if all(not self.exists[i] or m.loss < self.members[i].loss for i in range(size)):
                out.append(m.copy())
        return out


# ---------------------------------------------------------------------------------- tree utilities
def _nodes_with_parents(tree):
    """[(node, parent, which)] in pre-order; which = 0 (root), 1 (l), 2 (r)."""
    out, stack = [], [(tree, None, 0)]
    while stack:
        n, p, w = stack.pop()
        out.append((n, p, w))
        if n.degree == 2:
            stack.append((n.r, n, 2))
        if n.degree >= 1:
            stack.append((n.l, n, 1))
    return out


def _pick(rng, items):
    return items[int(rng.integers(0, len(items)))]


def mutate_factor(T, temperature, so, rng):
    """mutate_factor (src/MutationFunctions.jl), including its sign rule as written there."""
    bottom = 0.1
    max_change = so.perturbation_factor * temperature + 1 + bottom
    factor = T(T(max_change) ** T(rng.random()))
    if rng.random() >= 0.5:
        factor = T(1) / factor
    if rng.random() > so.probability_negate_constant:
        factor = factor * T(-1)
    return factor


def _new_op_node(arity, options, nfeatures, T, rng, carry=None):
    """A random operator node of `arity` with fresh random leaves, one of them (chosen uniformly)
    replaced by `carry` when given (append / insert / prepend_random_op)."""
    nops = options.operators.nops
    op = int(rng.integers(1, nops[arity - 1] + 1))
    kids = [make_random_leaf(nfeatures, T, rng) for _ in range(arity)]
    if carry is not None:
        kids[int(rng.integers(0, arity))] = carry
    return Node(op=op, l=kids[0], r=kids[1] if arity == 2 else None)


def _random_arity(options, rng):
    nops = options.operators.nops
    x = rng.random() * (nops[0] + nops[1])
    return 1 if (nops[0] > 0 and x <= nops[0]) else 2


def _rotate(tree, rng):
    """randomly_rotate_tree! (src/MutationFunctions.jl)."""
    def valid(n):
        return n.degree > 0 and any(c is not None and c.degree > 0 for c in (n.l, n.r))

    nodes = _nodes_with_parents(tree)
    roots = [(n, p, w) for (n, p, w) in nodes if valid(n)]
    if not roots:
        return tree
    at_root = rng.random() < 1.0 / len(roots)
    cands = [(n, p, w) for (n, p, w) in roots if n is not tree]
    if at_root or not cands:
        root, parent, widx, at_root = tree, None, 0, True
    else:
        root, parent, widx = _pick(rng, cands)
    kids = [i for i, c in ((1, root.l), (2, root.r)) if c is not None and c.degree > 0]
    pivot_idx = _pick(rng, kids)
    pivot = root.l if pivot_idx == 1 else root.r
    gc_idx = int(rng.integers(1, pivot.degree + 1))
    grand = pivot.l if gc_idx == 1 else pivot.r
    if pivot_idx == 1:
        root.l = grand
    else:
        root.r = grand
    if gc_idx == 1:
        pivot.l = root
    else:
        pivot.r = root
    if at_root:
        return pivot
    if widx == 1:
        parent.l = pivot
    else:
        parent.r = pivot
    return tree


def mutate(tree, choice, options, so, temperature, curmaxsize, nfeatures, T, rng):
    """One mutation (the ``mutate!`` methods of src/Mutate.jl:420-658); returns the new tree."""
    if choice == "mutate_constant":
        consts = [n for n in tree.preorder() if n.degree == 0 and n.constant]
        if consts:
            n = _pick(rng, consts)
            n.val = T(T(n.val) * mutate_factor(T, temperature, so, rng))
        return tree
    if choice == "mutate_operator":
        ops = [n for n in tree.preorder() if n.degree != 0]
        if ops:
            n = _pick(rng, ops)
            n.op = int(rng.integers(1, options.operators.nops[n.degree - 1] + 1))
        return tree
    if choice == "mutate_feature":
        feats = [n for n in tree.preorder() if n.degree == 0 and not n.constant]
        if nfeatures > 1 and feats:
            n = _pick(rng, feats)
            n.feature = _pick(rng, [f for f in range(1, nfeatures + 1) if f != n.feature])
        return tree
    if choice == "swap_operands":
        bins = [n for n in tree.preorder() if n.degree == 2]
        if bins:
            n = _pick(rng, bins)
            n.l, n.r = n.r, n.l
        return tree
    if choice == "rotate_tree":
        return _rotate(tree, rng)
    if choice == "add_node":
        if rng.random() < 0.5:  # append_random_op: a random leaf becomes a new operator node
            leaf = _pick(rng, [n for n in tree.preorder() if n.degree == 0])
            leaf.set_node(_new_op_node(_random_arity(options, rng), options, nfeatures, T, rng))
            return tree
        return _new_op_node(_random_arity(options, rng), options, nfeatures, T, rng, carry=tree)  # prepend
    if choice == "insert_node":
        n = _pick(rng, tree.preorder())
        n.set_node(_new_op_node(_random_arity(options, rng), options, nfeatures, T, rng, carry=n.copy()))
        return tree
    if choice == "delete_node":
        if tree.degree == 0:
            return tree
        n, p, w = _pick(rng, [(n, p, w) for (n, p, w) in _nodes_with_parents(tree) if n.degree > 0])
        carry = n.l if (n.degree == 1 or rng.integers(0, 2) == 0) else n.r
        if p is None:
            return carry
        if w == 1:
            p.l = carry
        else:
            p.r = carry
        return tree
    if choice == "randomize":
        return gen_random_tree_fixed_size(int(rng.integers(1, curmaxsize + 1)), options, nfeatures, T, rng)
    return tree


def crossover_trees(t1, t2, rng):
    """crossover_trees (src/MutationFunctions.jl): swap a random subtree of each copy."""
    a, b = t1.copy(), t2.copy()
    na, pa, wa = _pick(rng, _nodes_with_parents(a))
    nb, pb, wb = _pick(rng, _nodes_with_parents(b))
    na_c, nb_c = na.copy(), nb.copy()
    if pa is None:
        a = nb_c
    elif wa == 1:
        pa.l = nb_c
    else:
        pa.r = nb_c
    if pb is None:
        b = na_c
    elif wb == 1:
        pb.l = na_c
    else:
        pb.r = na_c
    return a, b


def condition_mutation_weights(w, member, so, curmaxsize, nfeatures):
    """condition_mutation_weights! (src/Mutate.jl:101-160)."""
    w = dict(w)
    tree = member.tree
    if tree.degree == 0:
        for k in ("mutate_operator", "swap_operands", "delete_node", "simplify"):
            w[k] = 0.0
        if not tree.constant:
            w["optimize"] = 0.0
            w["mutate_constant"] = 0.0
        else:
            w["mutate_feature"] = 0.0
        return w
    nodes = tree.preorder()  # one traversal for both counts
    if not any(n.degree == 2 for n in nodes):
        w["swap_operands"] = 0.0
    w["mutate_constant"] *= min(8, sum(1 for n in nodes if n.degree == 0 and n.constant)) / 8.0
    if nfeatures <= 1:
        w["mutate_feature"] = 0.0
    if member.complexity >= curmaxsize:
        w["add_node"] = 0.0
        w["insert_node"] = 0.0
    if not so.should_simplify:
        w["simplify"] = 0.0
    return w


def sample_mutation(w, rng):
    """sample_mutation (src/MutationWeights.jl): one draw ∝ the conditioned weights."""
    keys = [k for k in MUTATIONS if k in w]
    total = sum(w[k] for k in keys)
    r, acc = rng.random() * total, 0.0
    for k in keys:
        acc += w[k]
        if r < acc:
            return k
    return next(k for k in reversed(keys) if w[k] > 0)


def tournament_selection_weights(options):
    """get_tournament_selection_weights (src/Population.jl:150-163): p (1-p)^k, k = 0..n-1."""
    n, p = options.tournament_selection_n, np.float32(options.tournament_selection_p)
    w = (p * (np.float32(1) - p) ** np.arange(n, dtype=np.float32)).astype(np.float64)
    return w / w.sum()


def best_of_sample(pop, stats, options, so, rng, tweights):
    """best_of_sample / _best_of_sample (src/Population.jl:84-134); ranking follows argmin_fast /
    bottomk_fast (src/Utils.jl:96-147): strict <, first index wins, NaN (and +Inf) never ranked, a
    missing place falls back to the first member."""
    n = min(options.tournament_selection_n, len(pop))
    members = [pop[i] for i in rng.choice(len(pop), size=n, replace=False)]
    if so.use_frequency_in_tournament:
        # adjusted_costs::Vector{L} (src/Population.jl:124-139): cost * exp(L(scaling) * L(freq)),
        # every operation in the loss type L (Float32 for Float32 data)
        L = type(members[0].cost) if isinstance(members[0].cost, np.floating) else np.float64
        scaling = L(so.adaptive_parsimony_scaling)
        arg = np.array([scaling * L(stats.normalized_frequencies[m.complexity - 1]
                                    if 0 < m.complexity <= options.maxsize else 0.0) for m in members], dtype=L)
        factor = host_exp(arg)
        costs = [L(m.cost) * factor[i] for i, m in enumerate(members)]
    else:
        costs = [m.cost for m in members]
    ranked = sorted((i for i in range(n) if costs[i] < math.inf), key=lambda i: (costs[i], i))
    place = 0 if options.tournament_selection_p == 1.0 else _draw(tweights, rng)
    return members[ranked[place]] if place < len(ranked) else members[0]


def host_exp(x):
    """exp in the array's own precision with the library's host code (src/Population.jl computes the
    tournament weights with Julia's exp in L; the library's Float32 exp is correctly rounded but for
    2^-40-close midpoints, as Julia's Float32 exp)."""
    import ctypes

    x = np.ascontiguousarray(x)
    out = np.empty_like(x)
    dt = _lib.SR_DTYPE_F32 if x.dtype == np.float32 else _lib.SR_DTYPE_F64
    _lib.check(_lib.lib.sr_host_unary(dt, b"exp", x.size, x.ctypes.data_as(ctypes.c_void_p),
                                      out.ctypes.data_as(ctypes.c_void_p)))
    return out


def _draw(weights, rng):
    """Index drawn with probability weights[i] (weights sum to 1): inverse CDF of one uniform."""
    cdf = np.cumsum(weights)
    return min(int(np.searchsorted(cdf, rng.random() * cdf[-1], side="right")), len(weights) - 1)


def replace_oldest(pop, babies):
    used = set()
    for b in babies:
        oldest = min((j for j in range(len(pop)) if j not in used), key=lambda j: pop[j].birth)
        used.add(oldest)
        pop[oldest] = b


def migrate(candidates, pop, frac, rng, birth=_next_birth):
    """migrate! (src/Migration.jl:15-37): Poisson(n * frac) members replaced by copies (newest birth)."""
    n = len(pop)
    k = min(int(rng.poisson(n * frac)), len(candidates), n)
    for loc in rng.integers(0, n, size=max(k, 0)):
        m = candidates[int(rng.integers(0, len(candidates)))].copy()
        m.birth = birth()
        pop[int(loc)] = m


def random_population_trees(n, options, nfeatures, T, rng, nlength=3):
    """Population(dataset; population_size, nlength=3): gen_random_tree(3) = three
    append_random_op on a constant-0 leaf (src/MutationFunctions.jl gen_random_tree)."""
    trees = []
    for _ in range(n):
        t = Node(val=T(0))
        for _ in range(nlength):
            leaf = _pick(rng, [x for x in t.preorder() if x.degree == 0])
            leaf.set_node(_new_op_node(_random_arity(options, rng), options, nfeatures, T, rng))
        trees.append(t)
    return trees


# ---------------------------------------------------------------------------------- the search
@dataclass
class SearchResult:
    hall_of_fame: HallOfFame
    pareto_frontier: list
    populations: list
    iterations: int
    wall_s: float
    s_r_cycles: int
    num_evals: float
    device_calls: int


class _Plan:
    __slots__ = ("kind", "island", "parent", "parent2", "tree", "tree2", "slot", "temperature")

    def __init__(self, kind, island, parent=None, parent2=None, tree=None, tree2=None, slot=-1, temperature=1.0):
        self.kind, self.island, self.parent, self.parent2 = kind, island, parent, parent2
        self.tree, self.tree2, self.slot, self.temperature = tree, tree2, slot, temperature


def _costs(losses, sizes, ds, options):
    """loss_to_cost (src/LossFunctions.jl:170-190) over a batch: loss / normalization +
    L(size * parsimony::Float32), in the loss type as the scalar version computes it."""
    full = getattr(ds, "full", ds)
    L = losses.dtype.type
    base = L(full.baseline_loss)
    norm = base if (base >= L(0.01) and full.use_baseline) else L(0.01)
    pars = (np.asarray(sizes, dtype=np.float32) * np.float32(options.parsimony)).astype(losses.dtype)
    with np.errstate(over="ignore", invalid="ignore"):
        return (losses / norm + pars).astype(losses.dtype)  # costs are L, as PopMember.cost


def _accept(pl, after_cost, new_size, snap, maxsize, so, rng):
    """next_generation's acceptance test (src/Mutate.jl:273-317): NaN rejected; annealing
    exp(-delta / (T * alpha)); adaptive-parsimony frequency ratio; reject when prob < rand()."""
    if math.isnan(after_cost):
        return False
    prob = 1.0
    if so.annealing:
        # delta = after_cost - before_cost in L, then promoted against the Float64 temperature
        L = type(pl.parent.cost) if isinstance(pl.parent.cost, np.floating) else np.float64
        with np.errstate(over="ignore", invalid="ignore"):
            delta = float(L(after_cost) - L(pl.parent.cost))
        if pl.temperature > 0:
            with np.errstate(over="ignore", invalid="ignore"):
                prob *= float(np.exp(-delta / (pl.temperature * so.alpha)))
        else:
            prob *= 0.0 if delta > 0 else 1.0
    if so.use_frequency:
        old_size = pl.parent.complexity
        of = snap.normalized_frequencies[old_size - 1] if 0 < old_size <= maxsize else 1e-6
        nf = snap.normalized_frequencies[new_size - 1] if 0 < new_size <= maxsize else 1e-6
        prob *= of / nf
    return not (prob < rng.random())


def _torch_comm():
    """(rank, world, allgather_object) of the default torch.distributed group, or None."""
    try:
        import torch.distributed as tdist
    except ImportError:  # pragma: no cover
        return None
    if not (tdist.is_available() and tdist.is_initialized()) or tdist.get_world_size() == 1:
        return None
    world = tdist.get_world_size()

    def allgather(obj):
        out = [None] * world
        tdist.all_gather_object(out, obj)
        return out

    return tdist.get_rank(), world, allgather


def equation_search(X=None, y=None, *, niterations=10, options, weights=None, search_options=None, seed=0,
                    verbosity=0, dataset=None, distributed=False, _score_fn=None):
    """Batched-island ``equation_search`` on the device scoring path -> SearchResult.

    distributed=True (torch.distributed initialised, one process per GPU; SURVEY §8(e) island
    sharding): island i lives on rank i % world; every rank scores only its islands' children (one
    batched launch per round on its own GPU) and after each iteration the ranks all-gather their
    islands (members + best-seen) and replay the head node's island-by-island bookkeeping — running
    statistics, hall of fame, Pareto frontier — identically; migration into island i is done by its
    owner with the island's own random stream.  Random streams and birth counters are per island, so
    with constant optimisation off the result equals the single-process search's (tested); the
    constant-optimisation perturbations come from a per-rank stream.
    ``_score_fn(trees, dataset) -> (costs, losses)`` replaces the device scorer (CPU tests only)."""
    so = search_options or SearchOptions()
    comm = _torch_comm() if distributed else None
    rank, world, allgather = comm if comm else (0, 1, None)
    if dataset is None:
        dataset = Dataset(np.asarray(X), np.asarray(y), weights=weights)
    if _score_fn is None:
        update_baseline_loss_(dataset, options)
    else:  # update_baseline_loss! through the injected scorer
        dataset.use_baseline, dataset.baseline_loss = True, dataset.dtype.type(1)
        bl = _score_fn([Node(val=dataset.dtype.type(0))], dataset)[1][0]
        if np.isfinite(bl):
            dataset.baseline_loss = dataset.dtype.type(bl)
        else:
            dataset.use_baseline, dataset.baseline_loss = False, dataset.dtype.type(1)
    T = dataset.dtype.type
    nfeatures = dataset.nfeatures
    npop = options.populations
    owned = [i for i in range(npop) if i % world == rank]
    rngs = [np.random.default_rng([seed, i]) for i in range(npop)]
    births = [_Counter() for _ in range(npop)]  # birth order per island (replace_oldest compares within one)
    head_rng = np.random.default_rng([seed, 1_000_003, rank])
    maxsize = options.maxsize
    tweights = tournament_selection_weights(options)
    calls = [0]
    w_base = {k: v for k, v in so.mutation_weights.items() if k in MUTATIONS}

    def score(trees, ds):
        if not trees:
            return np.zeros(0), np.zeros(0)
        calls[0] += 1
        if _score_fn is not None:
            return _score_fn(trees, ds)
        tb = flatten_trees(trees, dataset.dtype)  # one flattening: the batch and the complexities
        losses, _ = eval_loss_batch(tb, ds, options)
        return _costs(losses, tb.tree_sizes(), ds, options), losses

    def exchange(pops, best_seen=None):
        """All-gather the owned islands (members, best-seen) so every rank holds all of them."""
        if world == 1:
            return
        mine = {i: (pops[i], None if best_seen is None else (best_seen[i].members, best_seen[i].exists))
                for i in owned}
        for part in allgather(mine):
            for i, (members, bs) in part.items():
                if i % world == rank:
                    continue
                pops[i] = members
                if best_seen is not None:
                    best_seen[i].members, best_seen[i].exists = bs

    # initial populations: one batched scoring launch for every (owned) island
    init = {i: random_population_trees(options.population_size, options, nfeatures, T, rngs[i]) for i in owned}
    flat = [t for i in owned for t in init[i]]
    c, l = score(flat, dataset)
    pops, k = [None] * npop, 0
    for i in owned:
        pop = []
        for t in init[i]:
            pop.append(PopMember(t, c[k], l[k], t.count_nodes(), birth=births[i]()))
            k += 1
        pops[i] = pop
    exchange(pops)
    stats = RunningSearchStatistics(maxsize)
    hof = HallOfFame(maxsize)
    best_sub_pops = [sorted(p, key=lambda m: m.cost)[: so.topn] for p in pops]
    num_evals = float(len(flat))
    t0 = time.perf_counter()
    total_cycles = niterations * npop
    cycles_done = 0
    for it in range(niterations):
        fraction_elapsed = cycles_done / max(1, total_cycles)
        curmaxsize = maxsize  # get_cur_maxsize (src/SearchUtils.jl:657-671)
        if so.warmup_maxsize_by > 0 and fraction_elapsed <= so.warmup_maxsize_by:
            curmaxsize = 3 + int((maxsize - 3) * fraction_elapsed / so.warmup_maxsize_by)
        snap = stats.copy()
        snap.normalize_frequencies()
        ds_iter = batch(dataset, options.batch_size, head_rng) if options.batching else dataset
        best_seen = [HallOfFame(maxsize) for _ in range(npop)]
        ncyc = options.ncycles_per_iteration
        temps = np.linspace(1.0, 0.0 if so.annealing else 1.0, ncyc) if ncyc > 1 else np.array([1.0])
        n_evol = math.ceil(options.population_size / options.tournament_selection_n)
        for temperature in temps:
            for _ in range(n_evol):
                plans, pending = [], []
                for i in owned:  # host: every island selects and mutates (or crosses over)
                    rng, pop = rngs[i], pops[i]
                    if rng.random() > so.crossover_probability:
                        allstar = best_of_sample(pop, snap, options, so, rng, tweights)
                        w = condition_mutation_weights(w_base, allstar, so, curmaxsize, nfeatures)
                        choice = sample_mutation(w, rng)
                        if choice in ("do_nothing", "simplify", "optimize"):
                            plans.append(_Plan("keep", i, allstar))  # return_immediately with the parent's cost
                            continue
                        tree = None
                        for _attempt in range(10):
                            cand = mutate(allstar.tree.copy(), choice, options, so, temperature, curmaxsize,
                                          nfeatures, T, rng)
                            if check_constraints(cand, options, curmaxsize):
                                tree = cand
                                break
                        if tree is None:
                            plans.append(_Plan("reject", i, allstar))
                            continue
                        plans.append(_Plan("mut", i, allstar, tree=tree, slot=len(pending),
                                           temperature=float(temperature)))
                        pending.append(tree)
                    else:
                        a1 = best_of_sample(pop, snap, options, so, rng, tweights)
                        a2 = best_of_sample(pop, snap, options, so, rng, tweights)
                        kids = None
                        for _try in range(11):
                            c1, c2 = crossover_trees(a1.tree, a2.tree, rng)
                            if check_constraints(c1, options, curmaxsize) and check_constraints(c2, options, curmaxsize):
                                kids = (c1, c2)
                                break
                        if kids is None:
                            plans.append(_Plan("reject", i, a1))
                            continue
                        plans.append(_Plan("cross", i, a1, a2, kids[0], kids[1], slot=len(pending)))
                        pending.extend(kids)
                costs, losses = score(pending, ds_iter)  # device: ONE batched eval_cost for all islands
                num_evals += len(pending) * ds_iter.dataset_fraction()
                for pl in plans:  # host: per-island acceptance, replacing the oldest member(s)
                    i = pl.island
                    rng, pop, born = rngs[i], pops[i], births[i]
                    if pl.kind == "reject":
                        if not so.skip_mutation_failures:
                            baby = pl.parent.copy()
                            baby.birth, baby.parent = born(), pl.parent.ref
                            replace_oldest(pop, [baby])
                        continue
                    if pl.kind == "keep":
                        p = pl.parent
                        replace_oldest(pop, [PopMember(p.tree.copy(), p.cost, p.loss, p.complexity, parent=p.ref,
                                                       birth=born())])
                        continue
                    if pl.kind == "cross":
                        j = pl.slot
                        b1 = PopMember(pl.tree, costs[j], losses[j], pl.tree.count_nodes(), parent=pl.parent.ref,
                                       birth=born())
                        b2 = PopMember(pl.tree2, costs[j + 1], losses[j + 1], pl.tree2.count_nodes(),
                                       parent=pl.parent2.ref, birth=born())
                        replace_oldest(pop, [b1, b2])
                        continue
                    j = pl.slot
                    new_size = pl.tree.count_nodes()
                    if _accept(pl, costs[j], new_size, snap, maxsize, so, rng):
                        replace_oldest(pop, [PopMember(pl.tree, costs[j], losses[j], new_size, parent=pl.parent.ref,
                                                       birth=born())])
                    elif not so.skip_mutation_failures:
                        baby = pl.parent.copy()
                        baby.birth, baby.parent = born(), pl.parent.ref
                        replace_oldest(pop, [baby])
            for i in owned:
                best_seen[i].update(pops[i], options, maxsize)
        # optimize_and_simplify_population: one batched constant optimisation for all (owned) islands
        if options.should_optimize_constants:
            sel = []
            for i in owned:
                do_opt = rngs[i].random(len(pops[i])) < options.optimizer_probability
                sel.extend((i, j) for j in np.nonzero(do_opt)[0] if pops[i][j].tree.count_constants() > 0)
            if sel:
                trees = [pops[i][j].tree for i, j in sel]
                new_tb, new_losses, improved, evals = optimize_constants_batch(
                    flatten_trees(trees, dataset.dtype), ds_iter, options, head_rng)
                calls[0] += 1
                num_evals += float(np.sum(evals))
                co, consts = new_tb.constant_offsets(), new_tb.get_constants()
                for k, (i, j) in enumerate(sel):
                    if not improved[k]:
                        continue
                    m = pops[i][j]
                    cnodes = [n for n in m.tree.preorder() if n.degree == 0 and n.constant]
                    for n, v in zip(cnodes, consts[co[k]:co[k + 1]]):
                        n.val = T(v)
                    m.loss = float(new_losses[k])
                    m.cost = float(loss_to_cost(T(new_losses[k]), dataset.use_baseline, dataset.baseline_loss,
                                                m.tree, options, m.complexity))
                    m.birth = births[i]()
        if options.batching:  # finalize_costs (src/Population.jl:182-196): re-score on the full data
            flat = [m for i in owned for m in pops[i]]
            c, l = score([m.tree for m in flat], dataset)
            for m, cc, ll in zip(flat, c, l):
                m.cost, m.loss = float(cc), float(ll)
        for i in owned:
            for m in pops[i]:
                m.parent, m.ref = m.ref, _next_ref()
        exchange(pops, best_seen)  # every rank now holds every island of this iteration
        for i in range(npop):  # head node, island by island (the reference's order), on every rank
            best_sub_pops[i] = sorted(pops[i], key=lambda m: m.cost)[: so.topn]
            for m in pops[i]:
                stats.update_frequencies(m.complexity)
            hof.update(pops[i], options, maxsize)
            hof.update([m for m, e in zip(best_seen[i].members, best_seen[i].exists) if e], options, maxsize)
            dominating = hof.pareto_frontier()
            if i % world == rank:  # the owner migrates with the island's own stream
                if so.migration:
                    migrate([m for p in best_sub_pops for m in p], pops[i], so.fraction_replaced, rngs[i],
                            births[i])
                if so.hof_migration and dominating:
                    migrate(dominating, pops[i], so.fraction_replaced_hof, rngs[i], births[i])
            cycles_done += 1
            stats.move_window()
        if verbosity and rank == 0:
            best = min((m for m in hof.members if m is not None), key=lambda m: m.loss)
            print(f"iteration {it + 1}/{niterations}: best loss {best.loss:.4g} (complexity {best.complexity})")
    exchange(pops)  # the final migrations
    if world > 1:
        num_evals = float(sum(allgather(num_evals)))
    wall = time.perf_counter() - t0
    return SearchResult(hof, hof.pareto_frontier(), pops, niterations, wall, niterations * npop, num_evals, calls[0])
