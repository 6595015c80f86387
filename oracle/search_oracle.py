"""TEST INFRASTRUCTURE ONLY — pure-Python restatement of the native search engine's algorithm.

An independent implementation (Node objects and Python ints, not the C++ pre-order arrays) of the
reference's search loop as ``csrc/sr_search.cpp`` runs it, with the same random-draw specification
(``csrc/sr_rng.h``) and the same lock-step round structure, so that the C++ engine and this module
must produce IDENTICAL populations and halls of fame from the same seed and the same scorer.  Each
function cites the reference code it restates:
  src/RegularizedEvolution.jl:12-160   reg_evol_cycle
  src/Mutate.jl:101-160, 174-356, 661-733   condition_mutation_weights!, next_generation,
                                             crossover_generation
  src/MutationFunctions.jl              every mutation (draw order per function)
  src/Population.jl:109-159             best_of_sample (bottomk_fast / argmin_fast, src/Utils.jl)
  src/SingleIteration.jl:19-139         s_r_cycle, optimize_and_simplify_population
  src/SymbolicRegression.jl:1040-1140   the head's per-island bookkeeping, migrate!, move_window!
Scores come from a caller-supplied ``loss_fn(trees, rows) -> losses`` (tests pass the C oracle): rows is
None (the full dataset) or, with ``batching``, one array of row indices per tree — its island's
minibatch, ``batch(dataset, batch_size)`` drawn per island per s_r_cycle (src/SingleIteration.jl:40;
src/Dataset.jl:303-304: rows with replacement).  Constant optimisation is not restated here (the tests
run with should_optimize_constants=False).
Only ``tests/`` import this module.
"""
from __future__ import annotations

import ctypes
import math

import numpy as np

M64 = (1 << 64) - 1


class Rng:
    """xoshiro256** with the draws of csrc/sr_rng.h."""

    def __init__(self, a, b):
        x = (a ^ (((b << 32) | (b >> 32)) & M64) ^ 0x5D6A7E1F3C2B4A99) & M64
        self.s = []
        for _ in range(4):
            x = (x + 0x9E3779B97F4A7C15) & M64
            z = x
            z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
            z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
            self.s.append(z ^ (z >> 31))

    @staticmethod
    def _rotl(x, k):
        return ((x << k) | (x >> (64 - k))) & M64

    def next(self):
        s = self.s
        r = (self._rotl((s[1] * 5) & M64, 7) * 9) & M64
        t = (s[1] << 17) & M64
        s[2] ^= s[0]
        s[3] ^= s[1]
        s[1] ^= s[2]
        s[0] ^= s[3]
        s[2] ^= t
        s[3] = self._rotl(s[3], 45)
        return r

    def uniform(self):
        return (self.next() >> 11) * 2.0 ** -53

    def uniform_f32(self):
        return np.float32((self.next() >> 40) * 2.0 ** -24)

    def uniform_t(self, T):
        return self.uniform_f32() if T == np.float32 else self.uniform()

    def below(self, n):
        return ((self.next() >> 32) * n) >> 32

    def coin(self):
        return (self.next() >> 63) != 0

    def normal(self):
        u1, u2 = self.uniform(), self.uniform()
        return math.sqrt(-2.0 * math.log(1.0 - u1)) * math.cos(6.283185307179586 * u2)


def _cexp(x):
    """C exp on doubles (Inf / 0 / NaN instead of Python's OverflowError)."""
    if math.isnan(x):
        return x
    try:
        return math.exp(x)
    except OverflowError:
        return math.inf


def host_unary(name, x, T):
    """Scalar op in T through the library's host code (the engine's own exp for the tournament
    weights and the Poisson draw; the ulp tests pin that code separately)."""
    from sr_amd import _lib

    a = np.array([x], dtype=T)
    out = np.empty_like(a)
    dt = _lib.SR_DTYPE_F32 if T == np.float32 else _lib.SR_DTYPE_F64
    _lib.check(_lib.lib.sr_host_unary(dt, name.encode(), 1, a.ctypes.data_as(ctypes.c_void_p),
                                      out.ctypes.data_as(ctypes.c_void_p)))
    return out[0]


# ------------------------------------------------------------------------ trees (sr_amd.Node)
def preorder(t):
    return t.preorder()


def nodes_with_parents(tree):
    """[(node, parent, which)] in pre-order; which = 0 root, 1 l, 2 r."""
    out, stack = [], [(tree, None, 0)]
    while stack:
        n, p, w = stack.pop()
        out.append((n, p, w))
        if n.degree == 2:
            stack.append((n.r, n, 2))
        if n.degree >= 1:
            stack.append((n.l, n, 1))
    return out


def sample(rng, items):
    return items[rng.below(len(items))] if items else None


class Spec:
    def __init__(self, options, so, nfeatures, T):
        from sr_amd import Node  # noqa: F401

        self.nfeatures = nfeatures
        self.nops = options.operators.nops
        self.unaops = options.operators.unaops
        self.binops = options.operators.binops
        self.maxdepth = options.maxdepth
        self.pf = float(np.float32(so.perturbation_factor))
        self.pnc = float(np.float32(so.probability_negate_constant))
        self.T = T


def make_leaf(sp, rng):
    from sr_amd import Node

    if rng.coin():
        return Node(val=sp.T(rng.normal()))
    return Node(feature=1 + rng.below(sp.nfeatures))


def scaled_arity(sp, rng):
    c1 = float(sp.nops[0])
    c2 = c1 + float(sp.nops[1])
    x = rng.uniform() * c2
    return 1 if (x > 0.0 and x <= c1) else 2


def make_node(arity, sp, rng):
    from sr_amd import Node

    op = 1 + rng.below(sp.nops[arity - 1])
    kids = [make_leaf(sp, rng) for _ in range(arity)]
    return Node(op=op, l=kids[0], r=kids[1] if arity == 2 else None)


def wrap_node(arity, carry, sp, rng):
    from sr_amd import Node

    slot = rng.below(arity)
    kids = [None] * arity
    for j in range(arity):
        if j != slot:
            kids[j] = make_leaf(sp, rng)
    kids[slot] = carry
    op = 1 + rng.below(sp.nops[arity - 1])
    return Node(op=op, l=kids[0], r=kids[1] if arity == 2 else None)


def mutate_factor(sp, temperature, rng):
    T = sp.T
    max_change = sp.pf * temperature + 1.0 + 0.1
    factor = T(math.pow(max_change, float(rng.uniform_t(T))))
    bigger = rng.coin()
    factor = factor if bigger else T(T(1) / factor)
    if rng.uniform() > sp.pnc:
        factor = T(factor * T(-1))
    return factor


def count_depth(t):
    return t.count_depth()


def check_constraints(t, sp, maxsize):
    return t.count_nodes() <= maxsize and count_depth(t) <= sp.maxdepth


def mutate(tree, choice, sp, temperature, curmax, rng):
    """One mutation on a copy (`tree`), returning the new tree."""
    T = sp.T
    if choice == "mutate_constant":
        n = sample(rng, [x for x in preorder(tree) if x.degree == 0 and x.constant])
        if n is not None:
            n.val = T(T(n.val) * mutate_factor(sp, temperature, rng))
        return tree
    if choice == "mutate_operator":
        n = sample(rng, [x for x in preorder(tree) if x.degree != 0])
        if n is not None:
            n.op = 1 + rng.below(sp.nops[n.degree - 1])
        return tree
    if choice == "mutate_feature":
        if sp.nfeatures <= 1:
            return tree
        n = sample(rng, [x for x in preorder(tree) if x.degree == 0 and not x.constant])
        if n is not None:
            k = rng.below(sp.nfeatures - 1)
            n.feature = k + 1 if k + 1 < n.feature else k + 2
        return tree
    if choice == "swap_operands":
        n = sample(rng, [x for x in preorder(tree) if x.degree > 1])
        if n is not None:
            rng.below(2)
            n.l, n.r = n.r, n.l
        return tree
    if choice == "rotate_tree":
        return rotate(tree, rng)
    if choice == "add_node":
        if rng.uniform() < 0.5:
            leaf = sample(rng, [x for x in preorder(tree) if x.degree == 0])
            leaf.set_node(make_node(scaled_arity(sp, rng), sp, rng))
            return tree
        return wrap_node(scaled_arity(sp, rng), tree, sp, rng)
    if choice == "insert_node":
        n = sample(rng, preorder(tree))
        n.set_node(wrap_node(scaled_arity(sp, rng), n.copy(), sp, rng))
        return tree
    if choice == "delete_node":
        if tree.degree == 0:
            return tree
        n, p, w = sample(rng, [(x, p, w) for (x, p, w) in nodes_with_parents(tree) if x.degree > 0])
        c = rng.below(n.degree)
        carry = n.l if c == 0 else n.r
        if p is None:
            return carry
        if w == 1:
            p.l = carry
        else:
            p.r = carry
        return tree
    if choice == "randomize":
        return gen_random_tree_fixed_size(1 + rng.below(curmax), sp, rng)
    raise AssertionError(choice)


def rotate(tree, rng):
    def valid(n):
        return n.degree > 0 and any(c is not None and c.degree > 0 for c in (n.l, n.r)[: n.degree])

    nodes = nodes_with_parents(tree)
    nvalid = sum(1 for (n, _, _) in nodes if valid(n))
    if nvalid == 0:
        return tree
    at_root = rng.uniform() < 1.0 / nvalid
    if at_root:
        root, parent, widx = tree, None, 0
    else:
        root, parent, widx = sample(rng, [(n, p, w) for (n, p, w) in nodes if n is not tree and valid(n)])
    kids = [c for c in range(root.degree) if (root.l, root.r)[c].degree > 0]
    pc = kids[rng.below(len(kids))]
    pivot = (root.l, root.r)[pc]
    gc = rng.below(pivot.degree)
    grand = (pivot.l, pivot.r)[gc]
    if pc == 0:
        root.l = grand
    else:
        root.r = grand
    if gc == 0:
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


def crossover(t1, t2, rng):
    a, b = t1.copy(), t2.copy()
    na = nodes_with_parents(a)
    nb = nodes_with_parents(b)
    n1, p1, w1 = na[rng.below(len(na))]
    n2, p2, w2 = nb[rng.below(len(nb))]
    c1, c2 = n1.copy(), n2.copy()
    if p1 is None:
        a = c2
    elif w1 == 1:
        p1.l = c2
    else:
        p1.r = c2
    if p2 is None:
        b = c1
    elif w2 == 1:
        p2.l = c1
    else:
        p2.r = c1
    return a, b


def gen_random_tree_fixed_size(node_count, sp, rng):
    t = make_leaf(sp, rng)
    cur = 1
    while True:
        remaining = node_count - cur
        if remaining == 0:
            break
        limit = min(2, remaining)
        total = sum(sp.nops[:limit])
        if total == 0:
            break
        thresh = 1 + rng.below(total)
        arity, acc = limit, 0
        for k in range(1, limit):
            acc += sp.nops[k - 1]
            if thresh <= acc:
                arity = k
                break
        leaf = sample(rng, [x for x in preorder(t) if x.degree == 0])
        leaf.set_node(make_node(arity, sp, rng))
        cur += arity
    return t


def gen_random_tree(length, sp, rng):
    from sr_amd import Node

    t = Node(val=sp.T(0))
    for _ in range(length):
        leaf = sample(rng, [x for x in preorder(t) if x.degree == 0])
        leaf.set_node(make_node(scaled_arity(sp, rng), sp, rng))
    return t


# --------------------------------------------------------------- simplification (DE, restated)
def _fold(name, vals, T, degree):
    """op applied in T by the C oracle (a one-node constant tree), None when not finite."""
    from oracle import Oracle
    from sr_amd import Node, Options, flatten_trees

    if degree == 1:
        opts = Options(binary_operators=["+"], unary_operators=[name])
        tree = Node(op=1, l=Node(val=vals[0]))
    else:
        opts = Options(binary_operators=[name], unary_operators=[])
        tree = Node(op=1, l=Node(val=vals[0]), r=Node(val=vals[1]))
    out, complete = Oracle.from_options(opts).eval_tree_array(flatten_trees([tree], T), 0, np.zeros((1, 1), T))
    v = T(out[0])
    return v if (complete and np.isfinite(v)) else None


def simplify(tree, sp):
    T = sp.T

    def is_const(n):
        return n.degree == 0 and n.constant

    def fold(n):
        if n.degree == 0:
            return
        fold(n.l)
        if n.degree == 2:
            fold(n.r)
        kids = [n.l] if n.degree == 1 else [n.l, n.r]
        if not all(is_const(c) for c in kids):
            return
        vals = [T(c.val) for c in kids]
        if not all(np.isfinite(v) for v in vals):
            return
        name = sp.unaops[n.op - 1] if n.degree == 1 else sp.binops[n.op - 1]
        v = _fold(name, vals, T, n.degree)
        if v is None:
            return
        n.degree, n.constant, n.val, n.op, n.l, n.r = 0, True, v, 0, None, None

    def combine(n):
        if n.degree == 0:
            return n
        n.l = combine(n.l)
        if n.degree == 2:
            n.r = combine(n.r)
        if n.degree != 2:
            return n
        name = sp.binops[n.op - 1]
        top_const = is_const(n.l) or is_const(n.r)
        if top_const and name in ("*", "+"):
            if is_const(n.l):
                n.l, n.r = n.r, n.l
            top = T(n.r.val)
            below = n.l
            if below.degree == 2 and below.op == n.op:
                if is_const(below.l):
                    n = below
                    n.l.val = T(_binop(name, T(n.l.val), top))
                elif is_const(below.r):
                    n = below
                    n.r.val = T(_binop(name, T(n.r.val), top))
        if n.degree == 2 and sp.binops[n.op - 1] == "-" and (is_const(n.l) or is_const(n.r)):
            if is_const(n.l):
                r = n.r
                if r.degree == 2 and sp.binops[r.op - 1] == "-":
                    l = n.l
                    if is_const(r.l):
                        c = T(-T(T(l.val) - T(r.l.val)))
                        n.l = r.r
                        n.r = l
                        l.val = c
                    elif is_const(r.r):
                        c = T(T(l.val) + T(r.r.val))
                        n.r = r.l
                        l.val = c
            else:
                l = n.l
                if l.degree == 2 and sp.binops[l.op - 1] == "-":
                    r = n.r
                    if is_const(l.l):
                        c = T(T(l.l.val) - T(r.val))
                        n.r = l.r
                        n.l = r
                        r.val = c
                    elif is_const(l.r):
                        c = T(T(r.val) + T(l.r.val))
                        n.l = l.l
                        r.val = c
        return n

    fold(tree)
    return combine(tree)


def _binop(name, a, b):
    with np.errstate(all="ignore"):
        return {"+": a + b, "*": a * b, "-": a - b}[name]


# ------------------------------------------------------------------------ the search
class Member:
    __slots__ = ("tree", "cost", "loss", "birth", "ref", "parent", "complexity")

    def __init__(self, tree, cost, loss, complexity, birth, ref, parent=-1):
        self.tree, self.cost, self.loss = tree, cost, loss
        self.complexity, self.birth, self.ref, self.parent = complexity, birth, ref, parent

    def copy(self):
        return Member(self.tree.copy(), self.cost, self.loss, self.complexity, self.birth, self.ref, self.parent)


MUTATIONS = ("mutate_constant", "mutate_operator", "mutate_feature", "swap_operands", "rotate_tree", "add_node",
             "insert_node", "delete_node", "simplify", "randomize", "do_nothing", "optimize")


BATCH_KEY = 0x6261746368  # the minibatch streams' key (csrc/sr_search.cpp draw_batch)


def draw_batch(seed, iteration, island, npop, salt, batch_size, n_rows):
    """The rows of island `island`'s minibatch in iteration `iteration` (salt 0: its s_r_cycle, 1: its
    constant optimisation): batch_size rows with replacement from their own xoshiro256** stream."""
    r = Rng(seed ^ BATCH_KEY, (iteration * npop + island) * 2 + salt)
    return np.array([r.below(n_rows) for _ in range(batch_size)], dtype=np.int64)


class SearchOracle:
    def __init__(self, options, so, nfeatures, n_rows, T, seed, loss_fn):
        self.o, self.so, self.T = options, so, T
        self.sp = Spec(options, so, nfeatures, T)
        self.n_rows = n_rows
        self.seed = seed
        self.loss_fn = loss_fn
        npop = options.populations
        self.rngs = [Rng(seed, i) for i in range(npop)]
        self.births = [0] * npop
        self.refs = [0] * npop
        self.num_evals = 0.0
        self.calls = 0

    # bookkeeping counters
    def birth(self, i):
        self.births[i] += 1
        return self.births[i]

    def ref(self, i):
        self.refs[i] += 1
        return ((i + 1) << 40) | self.refs[i]

    def cost_of(self, loss, complexity):
        T = self.T
        norm = self.baseline if (self.baseline >= T(0.01) and self.use_baseline) else T(0.01)
        with np.errstate(all="ignore"):
            v = T(T(loss) / norm)
            return T(v + T(np.float32(np.float32(complexity) * np.float32(self.o.parsimony))))

    def score(self, trees, rows=None):
        if not trees:
            return [], []
        self.calls += 1
        losses = np.asarray(self.loss_fn(trees, rows), dtype=self.T)
        return list(losses), [self.cost_of(losses[k], trees[k].count_nodes()) for k in range(len(trees))]

    def normalized(self):
        s = 0.0
        for f in self.freq:
            s += f
        return [f / s for f in self.freq]

    def cur_maxsize_now(self):
        elapsed = self.total_cycles - self.cycles_remaining
        frac = np.float32(np.float32(elapsed) / np.float32(self.total_cycles))
        w = np.float32(self.so.warmup_maxsize_by)
        if w > 0 and frac <= w:
            return 3 + int(math.floor(np.float32(np.float32(self.o.maxsize - 3) * frac) / w))
        return self.o.maxsize

    # --------------------------------------------------------------- selection
    def tweights(self):
        p = np.float32(self.o.tournament_selection_p)
        return [np.float32(p * np.float32(math.pow(float(np.float32(1) - p), k)))
                for k in range(self.o.tournament_selection_n)]

    def best_of_sample(self, i):
        rng, pop = self.rngs[i], self.pops[i]
        T = self.T
        np_ = len(pop)
        n = min(self.o.tournament_selection_n, np_)
        idx = list(range(np_))
        for k in range(n):
            j = k + rng.below(np_ - k)
            idx[k], idx[j] = idx[j], idx[k]
        nf = self.snap[i]
        adj = []
        for k in range(n):
            m = pop[idx[k]]
            if self.so.use_frequency_in_tournament:
                scaling = T(self.so.adaptive_parsimony_scaling)
                f = T(nf[m.complexity - 1]) if 0 < m.complexity <= self.o.maxsize else T(0)
                with np.errstate(all="ignore"):
                    e = host_unary("exp", T(scaling * f), T)
                    adj.append(T(T(m.cost) * e))
            else:
                adj.append(T(m.cost))
        if np.float32(self.o.tournament_selection_p) == np.float32(1.0):
            place = 0
        else:
            w = self.tweights()
            total = np.float32(0)
            for v in w:
                total = np.float32(total + v)
            t = rng.uniform() * float(total)
            place, cw = 0, w[0]
            while float(cw) < t and place + 1 < len(w):
                place += 1
                cw = np.float32(cw + w[place])
        K = place + 1
        mv, mi = [T(np.inf)] * K, [0] * K
        for k in range(n):
            if adj[k] < mv[K - 1]:
                mv[K - 1], mi[K - 1] = adj[k], k
                for q in range(K - 1, 0, -1):
                    if mv[q] < mv[q - 1]:
                        mv[q], mv[q - 1] = mv[q - 1], mv[q]
                        mi[q], mi[q - 1] = mi[q - 1], mi[q]
        return pop[idx[mi[K - 1]]].copy()

    def condition(self, m, curmax):
        w = dict(zip(MUTATIONS, [float(self.so.mutation_weights.get(k, 0.0)) for k in MUTATIONS]))
        t = m.tree
        if t.degree == 0:
            for k in ("mutate_operator", "swap_operands", "delete_node", "simplify"):
                w[k] = 0.0
            if not t.constant:
                w["optimize"] = 0.0
                w["mutate_constant"] = 0.0
            else:
                w["mutate_feature"] = 0.0
            return w
        nodes = preorder(t)
        if not any(n.degree == 2 for n in nodes):
            w["swap_operands"] = 0.0
        w["mutate_constant"] *= min(8, sum(1 for n in nodes if n.degree == 0 and n.constant)) / 8.0
        if self.sp.nfeatures <= 1:
            w["mutate_feature"] = 0.0
        if m.complexity >= curmax:
            w["add_node"] = 0.0
            w["insert_node"] = 0.0
        if not self.so.should_simplify:
            w["simplify"] = 0.0
        return w

    def sample_mutation(self, w, rng):
        total = 0.0
        for k in MUTATIONS:
            total += w[k]
        r = rng.uniform() * total
        acc = 0.0
        for k in MUTATIONS:
            acc += w[k]
            if r < acc:
                return k
        for k in reversed(MUTATIONS):
            if w[k] > 0:
                return k
        return "do_nothing"

    def replace_oldest(self, i, b):
        pop = self.pops[i]
        k = 0
        for j in range(1, len(pop)):
            if pop[j].birth < pop[k].birth:
                k = j
        pop[k] = b

    def replace_two(self, i, b1, b2):
        pop = self.pops[i]
        k1 = 0
        for j in range(1, len(pop)):
            if pop[j].birth < pop[k1].birth:
                k1 = j
        k2 = 1 if k1 == 0 else 0
        for j in range(len(pop)):
            if j != k1 and pop[j].birth < pop[k2].birth:
                k2 = j
        pop[k1], pop[k2] = b1, b2

    # --------------------------------------------------------------- one lock-step round
    def round(self, temperature):
        o, so, T = self.o, self.so, self.T
        plans, pending = [], []
        for i in range(o.populations):
            rng = self.rngs[i]
            curmax = self.cur_maxsize[i]
            if rng.uniform() > float(np.float32(so.crossover_probability)):
                par = self.best_of_sample(i)
                w = self.condition(par, curmax)
                choice = self.sample_mutation(w, rng)
                if choice == "do_nothing":
                    plans.append(["keep", i, par])
                elif choice == "simplify":
                    plans.append(["simp", i, par, simplify(par.tree.copy(), self.sp)])
                elif choice == "optimize":
                    plans.append(["opt", i, par])
                else:
                    tree, ok = None, False
                    for _ in range(10):
                        tree = mutate(par.tree.copy(), choice, self.sp, temperature, curmax, rng)
                        ok = check_constraints(tree, self.sp, curmax)
                        if ok:
                            break
                    plans.append(["mut" if ok else "reject", i, par, tree])
            else:
                a1 = self.best_of_sample(i)
                a2 = self.best_of_sample(i)
                ok = False
                for _ in range(11):
                    c1, c2 = crossover(a1.tree, a2.tree, rng)
                    ok = check_constraints(c1, self.sp, curmax) and check_constraints(c2, self.sp, curmax)
                    if ok:
                        break
                plans.append(["cross" if ok else "cross_fail", i, a1, a2, c1, c2])
        prow = []  # each pending tree's island minibatch (batching)
        for pl in plans:
            if pl[0] == "mut":
                pl.append(len(pending))
                pending.append(pl[3])
                prow.append(pl[1])
            elif pl[0] == "cross":
                pl.append(len(pending))
                pending.extend([pl[4], pl[5]])
                prow.extend([pl[1], pl[1]])
        rows = [self.batch_rows[i] for i in prow] if self.o.batching else None
        losses, costs = self.score(pending, rows)
        frac = self.o.batch_size / self.n_rows if self.o.batching else 1.0
        self.num_evals += len(pending) * frac
        for pl in plans:
            kind, i = pl[0], pl[1]
            rng = self.rngs[i]
            if kind in ("keep", "simp"):
                par = pl[2]
                b = par.copy()
                if kind == "simp":
                    b.tree = pl[3]
                    b.complexity = b.tree.count_nodes()
                b.parent, b.ref, b.birth = par.ref, self.ref(i), self.birth(i)
                self.replace_oldest(i, b)
            elif kind == "opt":  # (no constants optimised by this restatement)
                self.replace_oldest(i, pl[2])
            elif kind == "reject":
                if not so.skip_mutation_failures:
                    par = pl[2]
                    b = par.copy()
                    b.parent, b.ref, b.birth = par.ref, self.ref(i), self.birth(i)
                    self.replace_oldest(i, b)
            elif kind == "cross_fail":
                if not so.skip_mutation_failures:
                    self.replace_two(i, pl[2], pl[3])
            elif kind == "cross":
                j = pl[6]
                b1 = Member(pl[4], costs[j], losses[j], pl[4].count_nodes(), 0, 0, pl[2].ref)
                b1.ref, b1.birth = self.ref(i), self.birth(i)
                b2 = Member(pl[5], costs[j + 1], losses[j + 1], pl[5].count_nodes(), 0, 0, pl[3].ref)
                b2.ref, b2.birth = self.ref(i), self.birth(i)
                self.replace_two(i, b1, b2)
            else:  # mut
                par, tree, j = pl[2], pl[3], pl[4]
                after = costs[j]
                accept = not np.isnan(after)
                if accept:
                    prob = 1.0
                    if so.annealing:
                        with np.errstate(all="ignore"):
                            delta = T(T(after) - T(par.cost))
                            # IEEE division (temperature reaches 0): +-Inf / NaN exponents as in C
                            x = float(np.float64(-float(delta)) / np.float64(temperature * float(np.float32(so.alpha))))
                        prob *= _cexp(x)
                    new_size = tree.count_nodes()
                    if so.use_frequency:
                        nf = self.snap[i]
                        of = nf[par.complexity - 1] if 0 < par.complexity <= o.maxsize else 1e-6
                        nw = nf[new_size - 1] if 0 < new_size <= o.maxsize else 1e-6
                        prob *= of / nw
                    accept = not (prob < rng.uniform())
                if accept:
                    b = Member(tree, after, losses[j], tree.count_nodes(), 0, 0, par.ref)
                    b.ref, b.birth = self.ref(i), self.birth(i)
                    self.replace_oldest(i, b)
                elif not so.skip_mutation_failures:
                    b = par.copy()
                    b.parent, b.ref, b.birth = par.ref, self.ref(i), self.birth(i)
                    self.replace_oldest(i, b)

    # --------------------------------------------------------------- iteration / head
    def start(self, niterations):
        from sr_amd import Node

        o, T = self.o, self.T
        npop = o.populations
        self.freq = [1.0] * o.maxsize
        self.hof = [None] * o.maxsize
        self.total_cycles = max(1, niterations * npop)
        self.cycles_remaining = self.total_cycles
        self.head_maxsize = self.cur_maxsize_now()
        self.snap = [self.normalized() for _ in range(npop)]
        self.cur_maxsize = [self.head_maxsize] * npop
        bl = np.asarray(self.loss_fn([Node(val=T(0))], None), dtype=T)[0]
        self.calls += 1
        self.baseline, self.use_baseline = (T(bl), True) if np.isfinite(bl) else (T(1), False)
        trees, who = [], []
        for i in range(npop):
            for _ in range(o.population_size):
                trees.append(gen_random_tree(3, self.sp, self.rngs[i]))
                who.append(i)
        losses, costs = self.score(trees)
        self.num_evals += len(trees)
        self.pops = [[] for _ in range(npop)]
        for t, i, l, c in zip(trees, who, losses, costs):
            self.pops[i].append(Member(t, c, l, t.count_nodes(), self.birth(i), self.ref(i)))
        self.best_sub = [self.best_sub_pop(p) for p in self.pops]

    def best_sub_pop(self, pop):
        def key(k):
            c = pop[k].cost
            return (1, 0.0) if np.isnan(c) else (0, float(c))
        order = sorted(range(len(pop)), key=key)  # stable
        return [pop[k] for k in order[: self.so.topn]]

    def iterate(self):
        o = self.o
        npop = o.populations
        self.best_seen = [[None] * o.maxsize for _ in range(npop)]
        if self.o.batching:  # one minibatch per island for this iteration's s_r_cycle
            it = getattr(self, "iteration", 0)
            self.batch_rows = [draw_batch(self.seed, it, i, npop, 0, self.o.batch_size, self.n_rows)
                               for i in range(npop)]
        ncyc = o.ncycles_per_iteration
        n_evol = -(-o.population_size // o.tournament_selection_n)
        for c in range(ncyc):
            temperature = (1.0 - c / (ncyc - 1) if self.so.annealing else 1.0) if ncyc > 1 else 1.0
            for _ in range(n_evol):
                self.round(temperature)
            for i in range(npop):
                for m in self.pops[i]:
                    s = m.complexity
                    bs = self.best_seen[i]
                    if 0 < s <= o.maxsize and (bs[s - 1] is None or m.cost < bs[s - 1].cost):
                        bs[s - 1] = m.copy()
        for i in range(npop):
            pop = self.pops[i]
            for _ in pop:
                self.rngs[i].uniform()  # do_optimization draws (no optimisation in this restatement)
            for m in pop:
                if self.so.should_simplify:
                    m.tree = simplify(m.tree, self.sp)
                    m.complexity = m.tree.count_nodes()
        if self.o.batching:
            # finalize_costs on the full dataset (src/Population.jl:182-196), and the best-seen members
            # re-scored likewise (_dispatch_s_r_cycle), in one call: every island's members, then its
            # best-seen by size
            ms = []
            for i in range(npop):
                ms.extend(self.pops[i])
                ms.extend(m for m in self.best_seen[i] if m is not None)
            losses, costs = self.score([m.tree for m in ms])
            for m, l, c in zip(ms, losses, costs):
                m.loss, m.cost = l, c
            self.num_evals += len(ms)
        for i in range(npop):
            for m in self.pops[i]:
                m.parent, m.ref = m.ref, self.ref(i)
        self.iteration = getattr(self, "iteration", 0) + 1

    def hof_update(self, m):
        s = m.complexity
        if not (0 < s <= self.o.maxsize) or not check_constraints(m.tree, self.sp, self.o.maxsize):
            return
        if self.hof[s - 1] is None or m.cost < self.hof[s - 1].cost:
            self.hof[s - 1] = m.copy()

    def pareto(self):
        out = []
        for s, m in enumerate(self.hof):
            if m is None:
                continue
            if not any(self.hof[q] is not None and m.loss >= self.hof[q].loss for q in range(s)):
                out.append(m)
        return out

    def migrate(self, cands, i, frac):
        pop, rng, T = self.pops[i], self.rngs[i], self.T
        n = len(pop)
        lam = np.float32(np.float32(n) * np.float32(frac))
        k = 0
        if lam != 0:
            L = host_unary("exp", np.float32(-lam), np.float32)
            p = np.float32(1)
            while p > L:
                k += 1
                p = np.float32(p * rng.uniform_f32())
            k -= 1
        k = min(k, len(cands), n)
        if k <= 0:
            return
        loc = [rng.below(n) for _ in range(k)]
        mig = [rng.below(len(cands)) for _ in range(k)]
        for q in range(k):
            m = cands[mig[q]].copy()
            m.birth = self.birth(i)
            pop[loc[q]] = m

    def move_window(self):
        f = self.freq
        s = 0.0
        for v in f:
            s += v
        if s <= 100000.0:
            return
        diff = s - 100000.0
        loops = 0
        while diff > 0:
            idx = [k for k in range(len(f)) if f[k] > 1.0]
            if not idx:
                break
            amount = min(diff / len(idx), min(f[k] for k in idx) - 1.0)
            for k in idx:
                f[k] -= amount
            total = amount * len(idx)
            diff -= total
            loops += 1
            if loops > 1000 or total < 1e-6:
                break

    def head(self):
        o, so = self.o, self.so
        for i in range(o.populations):
            self.cur_maxsize[i] = self.head_maxsize
            self.best_sub[i] = self.best_sub_pop(self.pops[i])
            for m in self.pops[i]:
                if 0 < m.complexity <= len(self.freq):
                    self.freq[m.complexity - 1] += 1.0
            for m in self.pops[i]:
                self.hof_update(m)
            for m in self.best_seen[i]:
                if m is not None:
                    self.hof_update(m)
            dom = self.pareto()
            if so.migration:
                self.migrate([m for p in self.best_sub for m in p], i, so.fraction_replaced)
            if so.hof_migration and dom:
                self.migrate(dom, i, so.fraction_replaced_hof)
            self.cycles_remaining -= 1
            self.snap[i] = self.normalized()
            self.head_maxsize = self.cur_maxsize_now()
            self.move_window()

    def run(self, niterations):
        self.start(niterations)
        for _ in range(niterations):
            self.iterate()
            self.head()
        return self
