"""GPU: the reference's loss fold near Float32 overflow (src/LossFunctions.jl:38-58).

LossFunctions' `mean(loss, x, y)` and `sum(loss, x, y, w; normalize=true)` fold the elementwise losses
left to right in T, so a complete tree whose losses are finite but whose running Float32 sum passes
floatmax scores `L(Inf)` in the reference.  The library decides that from bounds on its f64 sum, from a
+Inf loss or pair of losses in its tiles, and for the undecided band folds the losses in row order on
the device (csrc/sr_fold.h; sr_aux.hip: the segmented fold — segment sums, composed steps per
segment, a chain over the segments with row-by-row scans where the fold crosses a binade).  The oracle's "ref" accumulation is that sequential fold,
so every case here is compared with it: +Inf exactly where it is +Inf, and — for the trees folded in
order — the same Float32 bits.
"""
import numpy as np
import pytest

import sr_amd
from oracle import Oracle
from sr_amd import Dataset, Options, eval_loss_batch, flatten_trees, parse_expression

pytestmark = pytest.mark.gpu

OPTS = dict(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp", "log"])
M = 3.4028235677973366e38  # 2^128 - 2^103: the smallest sum that rounds to +Inf in Float32


def _device_and_ref(exprs, X, y, w=None):
    opts = Options(**OPTS)
    tb = flatten_trees([parse_expression(e, opts) for e in exprs], np.float32)
    loss, comp = eval_loss_batch(tb, Dataset(X, y, weights=w), opts)
    ref, rcomp = Oracle.from_options(opts).eval_loss_batch(tb, X, y, w, accum="ref", n_threads=8)
    f64, _ = Oracle.from_options(opts).eval_loss_batch(tb, X, y, w, accum="f64", n_threads=8)
    return loss, comp, ref, rcomp, f64


def test_verdict_cases_overflow_to_inf_at_2p20_rows():
    """VERDICT r3 missing #1: at 2^20 rows, y = 0, the reference's Float32 fold of x1 * 0.0 + 3.2e16 and
    of x1 * 2.0e16 overflows (complete, L(Inf)); an f64 sum gives 1.02e33 and 4.0e32."""
    n = 1 << 20
    rng = np.random.default_rng(0)
    X = rng.standard_normal((5, n)).astype(np.float32)
    y = np.zeros(n, dtype=np.float32)
    loss, comp, ref, rcomp, _ = _device_and_ref(["x1 * 0.0 + 3.2e16", "x1 * 2.0e16", "x1 * 1.0e15"], X, y)
    assert comp.all() and rcomp.all()
    assert np.isinf(ref[:2]).all() and np.isfinite(ref[2])
    assert np.isinf(loss[:2]).all(), loss
    assert np.isfinite(loss[2]) and abs(float(loss[2]) / float(ref[2]) - 1) < 1e-3


def test_tile_sum_and_pair_overflow():
    """Losses of 1e36: every tile's T sum overflows but no pair does (the device then folds in order);
    losses of 2.25e38: a pair sum is +Inf (the fold is +Inf without folding); both are +Inf."""
    n = 1 << 17
    X = np.random.default_rng(1).standard_normal((5, n)).astype(np.float32)
    y = np.zeros(n, dtype=np.float32)
    ctx = sr_amd.get_context()
    for expr, folded in (("x1 * 0.0 + 1.0e18", 1), ("x1 * 0.0 + 1.5e19", 0)):
        loss, comp, ref, rcomp, _ = _device_and_ref([expr], X, y)
        assert comp[0] and rcomp[0] and np.isinf(ref[0]) and np.isinf(loss[0]), (expr, loss, ref)
        assert ctx.last_fold_trees() == folded, expr


@pytest.mark.parametrize("n", [1 << 17, 1 << 20])
def test_band_trees_fold_bit_exact(n):
    """x1 * c with Σ (c x1)^2 within +-0.7 % of the overflow threshold: the bounds cannot decide, the
    device folds in row order and must return the reference's Float32 fold / n bit for bit (and +Inf
    exactly where it overflows)."""
    rng = np.random.default_rng(2)
    X = rng.standard_normal((5, n)).astype(np.float32)
    y = np.zeros(n, dtype=np.float32)
    s2 = float(np.sum(X[0].astype(np.float64) ** 2))
    # (inside the band the bounds leave open at 2^17 rows: S in [M / 1.0078, 1.0078 M])
    fracs = [0.993, 0.996, 0.999, 1.0, 1.0005, 1.001, 1.004, 1.007]
    exprs = [f"x1 * {float(np.float32(np.sqrt(M * f / s2)))!r}" for f in fracs]
    loss, comp, ref, rcomp, f64 = _device_and_ref(exprs, X, y)
    assert comp.all() and rcomp.all()
    assert sr_amd.get_context().last_fold_trees() > 0
    assert np.array_equal(np.isinf(loss), np.isinf(ref)), (loss, ref)
    fin = np.isfinite(ref)
    assert np.array_equal(loss[fin].view(np.uint32), ref[fin].view(np.uint32)), (loss[fin], ref[fin])
    # the oracle's f64-accumulated loss takes its overflow verdict from the same fold
    assert np.array_equal(np.isinf(f64), np.isinf(ref))
    assert np.isinf(ref).any() and fin.any(), "the band should hold both verdicts"


def test_stagnating_fold_with_ties_weighted():
    """A fold that stagnates and rounds half-way cases to even: a first loss just under floatmax, then
    losses of exactly one and one half ulp of the running value (weights 1 and 0.5), in order.  The
    device's in-order fold (its binade-by-binade scan) must give the reference's fold bit for bit."""
    n = 1 << 17
    X = np.zeros((5, n), dtype=np.float32)
    X[0, 0] = np.float32(np.sqrt(3.39e38))
    X[0, 1:] = np.float32(2.0 ** 52)  # loss 2^104: one ulp of a value in [2^127, 2^128)
    y = np.zeros(n, dtype=np.float32)
    w = np.ones(n, dtype=np.float32)
    w[1::3] = np.float32(0.5)          # w * loss = 2^103: a tie, rounded to even
    for weights in (None, w):
        for x0 in (np.sqrt(3.39e38), np.sqrt(3.395e38), np.sqrt(3.37e38)):
            X[0, 0] = np.float32(x0)
            loss, comp, ref, rcomp, _ = _device_and_ref(["x1", "x1 * 1.0"], X, y, weights)
            assert comp.all() and rcomp.all()
            assert np.array_equal(np.isinf(loss), np.isinf(ref)), (x0, weights is None, loss, ref)
            fin = np.isfinite(ref)
            assert np.array_equal(loss[fin].view(np.uint32), ref[fin].view(np.uint32)), (x0, loss, ref)


def test_population_with_huge_predictions_matches_reference_fold():
    """A random population whose constants are scaled up (many trees near the overflow threshold):
    every complete tree is +Inf exactly where the reference's fold is, flags bit-exact."""
    opts = Options(**OPTS)
    n = 1 << 17
    rng = np.random.default_rng(3)
    X = rng.standard_normal((5, n)).astype(np.float32)
    y = (X[0] ** 2).astype(np.float32)
    trees = sr_amd.gen_random_population(3000, opts, 5, max_size=20, seed=3)
    for t in trees:  # one constant per tree scaled towards the overflow band
        c = sr_amd.get_scalar_constants(t)
        if c.size:
            c[0] *= 10.0 ** rng.uniform(14, 19)
            sr_amd.set_scalar_constants(t, c)
    tb = flatten_trees(trees, np.float32)
    loss, comp = eval_loss_batch(tb, Dataset(X, y), opts)
    ref, rcomp = Oracle.from_options(opts).eval_loss_batch(tb, X, y, accum="ref", n_threads=8)
    assert np.array_equal(comp, rcomp)
    assert np.array_equal(np.isinf(loss[comp]), np.isinf(ref[comp]))


def _fold_with_seg(tb, ds, opts, seg):
    ctx = sr_amd.get_context()
    ctx.set_tuning("fold_seg", seg)
    try:
        loss, comp = eval_loss_batch(tb, ds, opts)
        return loss, comp, ctx.last_fold_info()
    finally:
        ctx.set_tuning("fold_seg", -1)


@pytest.mark.parametrize("weighted", [False, True])
def test_segmented_fold_equals_single_scan(weighted):
    """The segmented fold (round 5) against rounds 3-4's single workgroup scan and the oracle's
    sequential Float32 fold, bit for bit, at 2^20 rows, for segment lengths 8k / 16k (automatic) / 64k /
    one scan: band trees (most segments advance by their composed steps; the fold crosses binades in a
    few), weights whose Float32 sum is inexact (the reference divides by its pairwise sum(w) in T)."""
    n = 1 << 20
    rng = np.random.default_rng(7)
    X = rng.standard_normal((5, n)).astype(np.float32)
    y = np.zeros(n, dtype=np.float32)
    w = rng.uniform(0.1, 1.9, n).astype(np.float32) if weighted else None
    opts = Options(**OPTS)
    wf = 1.0 if w is None else float(np.mean(w.astype(np.float64)))
    s2 = float(np.sum(X[0].astype(np.float64) ** 2)) * wf
    fracs = [0.95, 0.97, 0.985, 0.995, 0.999, 1.0, 1.001, 1.003, 1.01, 1.02]
    exprs = [f"x1 * {float(np.float32(np.sqrt(M * f / s2)))!r}" for f in fracs]
    exprs += [f"cos(x2) * {float(np.float32(np.sqrt(M * 0.999 / n)))!r} + x1 * 1.0e17"]
    tb = flatten_trees([parse_expression(e, opts) for e in exprs], np.float32)
    ds = Dataset(X, y, weights=w)
    ref, rcomp = Oracle.from_options(opts).eval_loss_batch(tb, X, y, w, accum="ref", n_threads=8)
    got = {}
    for seg in (0, 8192, -1, 65536):
        loss, comp, info = _fold_with_seg(tb, ds, opts, seg)
        assert comp.all() and rcomp.all()
        assert info[0] > 0, (seg, info)
        if seg > 0:
            assert info[2] == seg and info[1] < info[0] * (n // seg), (seg, info)  # most segments in O(1)
        got[seg] = loss
        assert np.array_equal(np.isinf(loss), np.isinf(ref)), (seg, loss, ref)
        fin = np.isfinite(ref)
        assert np.array_equal(loss[fin].view(np.uint32), ref[fin].view(np.uint32)), (seg, loss[fin], ref[fin])
    for seg in (8192, -1, 65536):
        assert np.array_equal(got[seg].view(np.uint32), got[0].view(np.uint32)), seg
