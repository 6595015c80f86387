"""GPU: every complete tree's loss is the reference's in-order loss fold (round 6).

The reference scores a complete tree with LossFunctions' `mean(loss, x, y)` / `sum(loss, x, y, w;
normalize=true)` (src/LossFunctions.jl:38-58): the elementwise losses folded left to right in T, then
divided in T.  Rounds 1-5 returned the f64 sum instead (~5e-4 relative off at 2^20 rows in Float32).
The library now computes the fold itself for every complete tree (csrc/sr_fold_dev.h): a plan from the
loss launch's f64 partials, each row block's composed steps (from the stored losses of a small call, or
from a FOLD-mode pass of the interpreter in a large one), and a walk over the row blocks.  So:

* the device loss equals a sequential Float32 fold (numpy's add.accumulate) of the device's OWN
  predictions bit for bit, for every complete tree, on both paths and at 2^20 rows;
* the two paths and the prediction-pass fallback give the same bits;
* against the oracle's `accum="ref"` (the C restatement of the reference's evaluator and fold): bit for
  bit for every tree without a transcendental, and for the rest within the libm bar.
"""
import numpy as np
import pytest

import sr_amd
from sr_amd import Dataset, Options, eval_loss_batch, eval_tree_array_batch, flatten_trees, gen_random_population

pytestmark = pytest.mark.gpu

OPTS = dict(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp", "log"])


def _data(n, seed=2, weighted=False):
    rng = np.random.default_rng(seed)
    X = rng.standard_normal((5, n)).astype(np.float32)
    y = (2 * np.cos(X[3]) + X[0] ** 2 - 2 + 0.1 * rng.standard_normal(n)).astype(np.float32)
    w = (0.25 + rng.random(n)).astype(np.float32) if weighted else None
    return X, y, w


def _jl_sum32(v):
    """Base.sum of a Float32 vector: mapreduce_impl's pairwise recursion, leaves of < 1024 folded in order."""
    def rec(lo, hi):
        if hi - lo < 1024:
            return np.add.accumulate(v[lo:hi + 1], dtype=np.float32)[-1]
        mid = lo + ((hi - lo) >> 1)
        return np.float32(rec(lo, mid) + rec(mid + 1, hi))
    return np.float32(rec(0, len(v) - 1))


def _np_fold_losses(pred, y, w=None):
    """LossFunctions' L2 mean (or weighted sum / sum(w)) of the given predictions, in Float32 and in row
    order: numpy's add.accumulate is a sequential left fold."""
    d = (pred - y).astype(np.float32)
    lo = d * d
    if w is not None:
        lo = (lo * w).astype(np.float32)
    total = np.add.accumulate(lo, dtype=np.float32)[-1]
    den = _jl_sum32(w) if w is not None else np.float32(len(y))
    return np.float32(total / den)


def _bits(a):
    return np.asarray(a, dtype=np.float32).view(np.uint32)


def _run(tb, ds, opts, **knobs):
    ctx = sr_amd.get_context()
    for k, v in knobs.items():
        ctx.set_tuning(k, v)
    try:
        loss, comp = eval_loss_batch(tb, ds, opts)
        info = ctx.last_ref_fold()
    finally:
        ctx.set_tuning("ref_fold", 1)
        ctx.set_tuning("fold_store_mb", 512)
        ctx.set_tuning("fold_delta_log2", 8)
        ctx.set_tuning("fold_debug_fail", 0)
    return loss, comp, info


@pytest.mark.parametrize("weighted", [False, True])
def test_fold_equals_sequential_fold_of_device_predictions(weighted):
    """Both paths (stored losses / FOLD mode) and a window so narrow that trees fall back to the
    prediction pass: every complete tree's loss is the sequential Float32 fold of its device
    predictions, bit for bit; ref_fold = 0 keeps the f64 sums (which differ in the last bits)."""
    n = 40_000
    X, y, w = _data(n, weighted=weighted)
    opts = Options(**OPTS)
    tb = flatten_trees(gen_random_population(1200, opts, 5, max_size=30, seed=7), np.float32)
    ds = Dataset(X, y, weights=w)
    l_s, c_s, i_s = _run(tb, ds, opts)
    assert i_s["path"] == 1 and i_s["folded"] > 300, i_s
    l_l, c_l, i_l = _run(tb, ds, opts, fold_store_mb=0)
    assert i_l["path"] == 2 and i_l["folded"] > 300, i_l
    # (every third tree through the fallback — the prediction pass and the segmented fold — as if its walk
    #  had left the plan's window; and a window of 2^-30 around the f64 prefix: far fewer slow segments)
    l_n, c_n, i_n = _run(tb, ds, opts, fold_store_mb=0, fold_delta_log2=30, fold_debug_fail=3)
    assert i_n["fallback"] > 100, i_n
    l_0, c_0, i_0 = _run(tb, ds, opts, ref_fold=0)
    assert i_0["path"] == 0
    for c in (c_l, c_n, c_0):
        assert np.array_equal(c, c_s)
    fin = c_s & np.isfinite(l_s)
    assert np.array_equal(_bits(l_s[fin]), _bits(l_l[fin]))
    assert np.array_equal(_bits(l_s[fin]), _bits(l_n[fin]))
    assert not np.array_equal(_bits(l_s[fin]), _bits(l_0[fin]))  # (the f64 sums: other last bits)
    pred, pcomp = eval_tree_array_batch(tb, ds, opts)
    idx = np.nonzero(fin)[0]
    want = np.array([_np_fold_losses(pred[t], y, w) for t in idx], dtype=np.float32)
    bad = idx[_bits(l_s[idx]) != _bits(want)]
    assert bad.size == 0, (bad[:5], l_s[bad[:5]], want[:5])


def test_fold_at_2p20_rows_c2_distribution():
    """C2's distribution at its full row count (FOLD-mode path): a 1,000-tree sample of the C2
    population generator, every complete tree's loss the sequential Float32 fold of its predictions."""
    n = 1 << 20
    X, y, _ = _data(n, seed=2)
    opts = Options(**OPTS)
    tb = flatten_trees(gen_random_population(1000, opts, 5, max_size=30, seed=1), np.float32)
    ds = Dataset(X, y)
    loss, comp, info = _run(tb, ds, opts)
    assert info["path"] == 2, info
    fin = comp & np.isfinite(loss)
    assert info["folded"] + info["fallback"] >= int(fin.sum()) - 5, (info, int(fin.sum()))
    idx = np.nonzero(fin)[0]
    rng = np.random.default_rng(0)
    pick = np.sort(rng.choice(idx, size=min(120, idx.size), replace=False))
    sub = tb.take(pick)
    pred, _ = eval_tree_array_batch(sub, ds, opts)
    want = np.array([_np_fold_losses(pred[k], y) for k in range(len(pick))], dtype=np.float32)
    assert np.array_equal(_bits(loss[pick]), _bits(want)), (loss[pick][:4], want[:4])
    # the f64 sum differs from the fold by ~5e-4 relative here (what rounds 1-5 returned)
    l64, _, _ = _run(tb, ds, opts, ref_fold=0)
    rel = np.abs(l64[fin].astype(np.float64) - loss[fin]) / np.abs(loss[fin].astype(np.float64))
    assert float(np.median(rel)) > 1e-5


def test_fold_vs_oracle_reference_accumulation():
    """Against the oracle's accum="ref" (the C restatement of DE's evaluator and of LossFunctions'
    fold): every complete tree built from + - * / only equals it bit for bit; the others (Float32
    cos / exp / log: last-bit libm differences) within 1e-4, most bit for bit."""
    from oracle import Oracle

    n = 30_000
    X, y, _ = _data(n, seed=5)
    opts = Options(**OPTS)
    tb = flatten_trees(gen_random_population(800, opts, 5, max_size=30, seed=3), np.float32)
    loss, comp, info = _run(tb, Dataset(X, y), opts)
    ref, rcomp = Oracle.from_options(opts).eval_loss_batch(tb, X, y, accum="ref", n_threads=8)
    assert np.array_equal(comp, rcomp)
    fin = comp & np.isfinite(ref)
    deg = np.asarray(tb.degree)
    offs = np.asarray(tb.offsets)
    arith = np.array([not np.any(deg[offs[t]:offs[t + 1]] == 1) for t in range(tb.n_trees)])
    sel = fin & arith
    assert sel.sum() > 50
    assert np.array_equal(_bits(loss[sel]), _bits(ref[sel]))
    # the rest within the tests' per-tree bar: 1e-4, or 4x the tree's spread under +-1-ulp libm
    # perturbations (a tree that amplifies last-bit libm differences: exp in a cancellation, ...)
    from parity_util import loss_tolerance
    tol, _, _, _ = loss_tolerance(Oracle.from_options(opts), tb, X, y)
    err = np.abs(loss.astype(np.float64) - ref.astype(np.float64))
    bad = np.nonzero(fin & ~(err <= tol))[0]
    assert bad.size == 0, [(int(k), float(loss[k]), float(ref[k]), float(tol[k])) for k in bad[:5]]
    assert float(np.mean(_bits(loss[fin]) == _bits(ref[fin]))) > 0.9


def _fold_np(l, dtype):
    f = dtype(l[0])
    for v in l[1:]:
        f = dtype(f + v)
    return f


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("n", [100, 256, 257, 3001, 40_000])
def test_short_views_and_the_serial_start(dtype, n):
    """The walk folds the first 256 rows one by one in hardware adds, then row blocks: views shorter
    than, equal to and just past that, a block wholly inside it (Float64 R4 tiles of 256 rows: round 6's
    bug read the next block's rows from a stale pass), and two paths of blocks."""
    from sr_amd import parse_expression

    opts = Options(binary_operators=["+", "*", "-", "/"], unary_operators=["cos", "exp"])
    rng = np.random.default_rng(n)
    X = rng.standard_normal((3, n)).astype(dtype)
    y = (X[0] * 2 + 0.1 * rng.standard_normal(n)).astype(dtype)
    tb = flatten_trees([parse_expression(e, opts) for e in ("3.2 * x1", "x1 * x2", "(x1 - x3) * 0.7")], dtype)
    loss, comp, info = _run(tb, Dataset(X, y), opts)
    assert info["path"] == 1 and info["folded"] == 3 and info["fallback"] == 0, info
    preds = [dtype(dtype(3.2) * X[0]), X[0] * X[1], (X[0] - X[2]) * dtype(0.7)]
    for k, p in enumerate(preds):
        d = (p - y).astype(dtype)
        want = dtype(_fold_np((d * d).astype(dtype), dtype) / dtype(n))
        assert loss[k] == want, (k, loss[k], want)


def test_stored_path_folds_drifted_runs_row_by_row():
    """With every loss kept (a small call), a run of blocks whose binade the plan mispredicted is folded
    row by row on the spot: a window of 2^-30 around the f64 prefix (every run the fold drifts out of)
    gives the default window's bits and no fallback."""
    n = 40_000
    X, y, _ = _data(n, seed=9)
    opts = Options(**OPTS)
    tb = flatten_trees(gen_random_population(600, opts, 5, max_size=30, seed=11), np.float32)
    ds = Dataset(X, y)
    l_s, c_s, i_s = _run(tb, ds, opts)
    l_n, c_n, i_n = _run(tb, ds, opts, fold_delta_log2=30)
    assert i_s["path"] == 1 and i_n["path"] == 1
    assert i_n["fallback"] == 0 and i_n["folded"] == i_s["folded"], (i_s, i_n)
    fin = c_s & np.isfinite(l_s)
    assert np.array_equal(_bits(l_s[fin]), _bits(l_n[fin]))


def test_constant_trees_fold_without_fallback_at_2p20_rows():
    """Trees whose losses hardly vary ((c - y)^2 with a huge constant c) drift from the f64 prefix by up
    to ~1 % at 2^20 rows (every step rounds the same way): the plan widens their window, and the
    FOLD-mode path folds them with no fallback, bit for bit."""
    from sr_amd import parse_expression

    n = 1 << 20
    X, y, _ = _data(n, seed=2)
    opts = Options(**OPTS)
    exprs = ["exp(exp(exp(1.0642476)))", "exp(exp(2.2194602))", "(exp(exp(1.8301688)) / 0.39640316)",
             "exp(exp(2.477696)) + (x2 - cos(0.019))", "x1 + 3000.0", "(x2 * 0.001) + 77.5"]
    tb = flatten_trees([parse_expression(e, opts) for e in exprs], np.float32)
    ds = Dataset(X, y)
    loss, comp, info = _run(tb, ds, opts, fold_store_mb=0)
    assert info["path"] == 2 and info["fallback"] == 0 and info["folded"] == int(comp.sum()), info
    pred, _ = eval_tree_array_batch(tb, ds, opts)
    for k in range(tb.n_trees):
        if comp[k]:
            want = _np_fold_losses(pred[k], y)
            assert _bits(loss[k]) == _bits(want), (exprs[k], loss[k], want)


def test_fold_rows_max_keeps_the_f64_sum_past_it():
    """Calls longer than fold_rows_max (2^24 rows by default: C4's 2^26-row Float32 fold stalls far below
    the exact mean) keep the f64 sums; ref_fold_info says path 0."""
    n = 20_000
    X, y, _ = _data(n, seed=4)
    opts = Options(**OPTS)
    tb = flatten_trees(gen_random_population(200, opts, 5, max_size=20, seed=5), np.float32)
    ds = Dataset(X, y)
    l1, c1, i1 = _run(tb, ds, opts)
    ctx = sr_amd.get_context()
    try:
        l0, c0, i0 = _run(tb, ds, opts, fold_rows_max=n - 1)
    finally:
        ctx.set_tuning("fold_rows_max", 1 << 24)
    l2, c2, i2 = _run(tb, ds, opts, ref_fold=0)
    assert i1["path"] == 1 and i0["path"] == 0
    assert np.array_equal(c0, c1)
    fin = c1 & np.isfinite(l1)
    assert np.array_equal(_bits(l0[fin]), _bits(l2[fin]))  # exactly the ref_fold 0 results
