"""GPU: the in-launch partial reduction (the last workgroup of each tree group reduces it; an option,
`fused_reduce`, off by default: measured slower than the separate reduce launch).

A multi-row-block LOSS launch writes its per-(row block, tree) partials with write-through stores; the
workgroup whose counter add comes last reduces the group in `sr_reduce_partials_kernel`'s order.  Its
results must be bit-identical to the separate reduce launch (`fused_reduce` = 0) for every shape the
search and the headline use: a few trees over many row blocks (C3's scoring calls), thousands of trees
on both kernel builds and both pipeline chunks, Float64 with weights, several row views in one launch —
and stay identical over repeated calls (a stale read of another workgroup's partial would show up as
a changed sum under the uneven per-tree load of a random population).
"""
import numpy as np
import pytest

import sr_amd
from sr_amd import Dataset, Options, eval_loss_batch, eval_loss_batch_views, flatten_trees, gen_random_population

pytestmark = pytest.mark.gpu

OPTS = dict(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp", "log"])


def _data(n, dtype, weighted, seed):
    rng = np.random.default_rng(seed)
    X = rng.standard_normal((5, n)).astype(dtype)
    y = (2 * np.cos(X[3]) + X[0] ** 2 - 2).astype(dtype)
    w = (0.5 + rng.random(n)).astype(dtype) if weighted else None
    return Dataset(X, y, weights=w)


def _both(fn):
    ctx = sr_amd.get_context()
    ctx.set_tuning("fused_reduce", 1 << 30)
    try:
        fused = fn()
        ctx.set_tuning("fused_reduce", 0)
        plain = fn()
    finally:
        ctx.set_tuning("fused_reduce", 0)  # (the default: a separate reduce launch)
    return fused, plain


@pytest.mark.parametrize("n_trees,n_rows,dtype,weighted", [
    (31, 100_000, np.float32, False),      # C3's scoring call
    (3000, 1 << 17, np.float32, False),    # both builds, two chunks
    (500, 50_000, np.float64, True),
])
def test_fused_reduce_equals_reduce_launch(n_trees, n_rows, dtype, weighted):
    opts = Options(**OPTS)
    ds = _data(n_rows, dtype, weighted, seed=n_trees)
    tb = flatten_trees(gen_random_population(n_trees, opts, 5, max_size=30, dtype=dtype, seed=n_trees), dtype)
    (lf, cf), (lp, cp) = _both(lambda: eval_loss_batch(tb, ds, opts))
    assert np.array_equal(cf, cp)
    assert np.array_equal(lf.view(np.uint8), lp.view(np.uint8))
    assert 0.05 < cf.mean() < 0.95
    ctx = sr_amd.get_context()
    ctx.set_tuning("fused_reduce", 1 << 30)
    try:
        for _ in range(5):  # repeated fused calls: the same bits every time
            l2, c2 = eval_loss_batch(tb, ds, opts)
            assert np.array_equal(c2, cf) and np.array_equal(l2.view(np.uint8), lf.view(np.uint8))
    finally:
        ctx.set_tuning("fused_reduce", 0)


def test_fused_reduce_views():
    opts = Options(**OPTS)
    ds = _data(60_000, np.float32, True, seed=9)
    tb = flatten_trees(gen_random_population(700, opts, 5, max_size=25, seed=9), np.float32)
    rng = np.random.default_rng(9)
    views = rng.integers(0, 60_000, (6, 30_000))
    tree_view = rng.integers(0, 6, tb.n_trees)
    (lf, cf), (lp, cp) = _both(lambda: eval_loss_batch_views(tb, ds, opts, tree_view, views))
    assert np.array_equal(cf, cp)
    assert np.array_equal(lf.view(np.uint8), lp.view(np.uint8))
