"""Random tree generators (reference src/MutationFunctions.jl:321-471).

They define the benchmark population: ``gen_random_tree_fixed_size`` is the generator the reference
uses for ``randomize_tree`` and initial populations.  Host-side only (mutation stays on the CPU).
"""
from __future__ import annotations

import numpy as np

from .node import Node


def sample_value(rng: np.random.Generator, dtype=np.float32):
    # sample_value(rng, T, _) = randn(rng, T)  (src/InterfaceDataTypes.jl:20)
    return dtype(rng.standard_normal())


def make_random_leaf(nfeatures: int, dtype, rng: np.random.Generator) -> Node:
    """50 % constant ~ randn(T), 50 % feature uniform in 1:nfeatures (src/MutationFunctions.jl:321-333)."""
    if rng.integers(0, 2) == 1:
        return Node(val=sample_value(rng, dtype))
    return Node(feature=int(rng.integers(1, nfeatures + 1)))


def _arity_picker(rng: np.random.Generator, remaining: int, nops) -> int:
    """src/MutationFunctions.jl:424-439: arity ∝ number of operators of that arity, capped by
    the remaining node budget."""
    D = len(nops)
    limit = min(D, remaining)
    total = sum(nops[:limit])
    if total == 0:
        return 0
    thresh = int(rng.integers(1, total + 1))
    acc = 0
    for k in range(1, limit):
        acc += nops[k - 1]
        if thresh <= acc:
            return k
    return limit


def _leaves(tree: Node):
    return [n for n in tree.preorder() if n.degree == 0]


def gen_random_tree_fixed_size(node_count: int, options, nfeatures: int, dtype=np.float32,
                               rng: np.random.Generator | None = None) -> Node:
    """src/MutationFunctions.jl:441-471: start from a random leaf, repeatedly replace a uniformly
    chosen leaf by an operator node with fresh random leaves until ``node_count`` is reached."""
    rng = rng or np.random.default_rng()
    tree = make_random_leaf(nfeatures, dtype, rng)
    cur_size = 1
    nops = options.operators.nops  # (n_unary, n_binary)
    while True:
        remaining = node_count - cur_size
        if remaining == 0:
            break
        arity = _arity_picker(rng, remaining, nops)
        if arity == 0:
            break
        leaves = _leaves(tree)
        leaf = leaves[int(rng.integers(0, len(leaves)))]
        op = int(rng.integers(1, nops[arity - 1] + 1))
        if arity == 1:
            new = Node(op=op, l=make_random_leaf(nfeatures, dtype, rng))
        else:
            l = make_random_leaf(nfeatures, dtype, rng)
            r = make_random_leaf(nfeatures, dtype, rng)
            new = Node(op=op, l=l, r=r)
        leaf.set_node(new)
        cur_size += arity
    return tree


def gen_random_population(n_trees: int, options, nfeatures: int, *, max_size: int = 30, dtype=np.float32,
                          seed: int = 1):
    """BASELINE C2 population: ``node_count ~ U{1..max_size}`` trees from the fixed-size generator."""
    rng = np.random.default_rng(seed)
    sizes = rng.integers(1, max_size + 1, size=n_trees)
    return [gen_random_tree_fixed_size(int(s), options, nfeatures, dtype, rng) for s in sizes]


def gen_random_batch(n_trees: int, options, nfeatures: int, *, max_size: int = 30, dtype=np.float32, seed: int = 1):
    """A TreeBatch of ``n_trees`` random trees (``node_count ~ U{1..max_size}``) from the library's native
    gen_random_tree_fixed_size (C ABI ``sr_gen_random_population``; the engine's generator and draws,
    one stream keyed by ``seed``) — the same distribution as ``gen_random_population`` at C speed."""
    import ctypes

    from . import _lib
    from .node import TreeBatch

    cap = int(n_trees) * int(max_size)
    offs = np.zeros(n_trees + 1, np.int64)
    deg, op, con = (np.zeros(max(cap, 1), np.uint8) for _ in range(3))
    feat = np.zeros(max(cap, 1), np.uint16)
    val = np.zeros(max(cap, 1), dtype)
    p = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    _lib.check(_lib.lib.sr_gen_random_population(
        _lib.SR_DTYPE_F32 if np.dtype(dtype) == np.float32 else _lib.SR_DTYPE_F64, int(n_trees), int(nfeatures),
        len(options.operators.unaops), len(options.operators.binops), int(max_size), int(seed), cap, p(offs), p(deg),
        p(op), p(feat), p(con), p(val)))
    nn = int(offs[-1])
    return TreeBatch(offs, deg[:nn].copy(), op[:nn].copy(), feat[:nn].copy(), con[:nn].copy(), val[:nn].copy())
