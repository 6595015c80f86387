"""Packed fast paths of the f32 interpreter are bit-identical to the full operations.

* ``a / b`` (csrc/sr_tile_impl.h ``sr_div_rows_f32``): the Newton/Markstein core of the library's
  correctly rounded division, two rows per packed instruction, taken when every row of the wave has
  |a|, |b| in [2^-40, 2^40]; otherwise the full division (operand scaling + special-case fixup).
  Julia's ``/`` on Float32 is IEEE division, so numpy's float32 division is the exact reference
  here: every output bit must match, in both paths and at the path boundary.
* ``exp`` (``sr_exp_rows_f32``): OCML's expf sequence without its range selects when every row of
  the wave has |x| <= 88.  The same values evaluated in a tile that is forced onto the full path
  (one row with |x| > 88) must give the same bits.
"""
import numpy as np
import pytest

from sr_amd import Options, eval_tree_array, parse_expression

pytestmark = pytest.mark.gpu


def _bits(a):
    return np.asarray(a, dtype=np.float32).view(np.uint32)


def _log_uniform(rng, n, lo_exp, hi_exp):
    mag = np.exp2(rng.uniform(lo_exp, hi_exp, n)).astype(np.float32)
    return np.where(rng.random(n) < 0.5, -mag, mag).astype(np.float32)


def _division_operands(seed):
    rng = np.random.default_rng(seed)
    n = 1 << 16
    a = _log_uniform(rng, n, -39.5, 39.5)
    b = _log_uniform(rng, n, -39.5, 39.5)
    # adversarial mantissas: all-ones / power-of-two / near-midpoint denominators, a = k*b +- ulp
    ones = np.float32(np.nextafter(np.float32(2), np.float32(0)))
    b[:512] = ones * np.exp2(rng.integers(-30, 30, 512)).astype(np.float32)
    b[512:1024] = np.exp2(rng.integers(-39, 39, 512)).astype(np.float32)
    k = rng.integers(1, 1 << 20, 512).astype(np.float32)
    a[1024:1536] = np.nextafter(k * b[1024:1536], np.float32(np.inf) * np.sign(rng.standard_normal(512)))
    # tiles that leave the fast range in one row (the full path), and magnitudes near its edges
    for t in range(6, 24, 3):
        s = t * 512
        a[s + 7] = np.float32(2.0 ** 45)
        b[s + 100] = np.float32(2.0 ** -47)
    edge = np.float32(2.0 ** 40)
    a[24 * 512: 25 * 512] = edge * np.float32(rng.uniform(0.5, 1.0, 512))
    b[25 * 512: 26 * 512] = np.float32(2.0 ** -40) * np.float32(rng.uniform(1.0, 2.0, 512))
    b[26 * 512: 26 * 512 + 3] = np.float32(2.0 ** -40), np.float32(2.0 ** 40), np.nextafter(np.float32(2.0 ** 40), np.float32(np.inf))
    # large and tiny finite quotients through the full path
    a[27 * 512: 27 * 512 + 64] = np.float32(1e25)
    b[27 * 512: 27 * 512 + 64] = np.float32(3e-7)
    a[28 * 512: 28 * 512 + 64] = np.float32(1e-25)
    b[28 * 512: 28 * 512 + 64] = np.float32(7e7)
    return a, b


@pytest.mark.parametrize("expr", ["x1 / x2", "x2 / x1", "(x1 * 1.5) / x2", "x1 / (x2 + 0.25)", "2.5 / x1",
                                  "(x1 - x2) / (x1 * x2)"])
def test_division_bit_exact_vs_ieee(expr):
    a, b = _division_operands(3)
    opts = Options(binary_operators=["+", "-", "*", "/"], unary_operators=[])
    tree = parse_expression(expr, opts)
    x1, x2 = a, b
    f32 = np.float32
    with np.errstate(all="ignore"):
        want = {
            "x1 / x2": x1 / x2,
            "x2 / x1": x2 / x1,
            "(x1 * 1.5) / x2": (x1 * f32(1.5)) / x2,
            "x1 / (x2 + 0.25)": x1 / (x2 + f32(0.25)),
            "2.5 / x1": f32(2.5) / x1,
            "(x1 - x2) / (x1 * x2)": (x1 - x2) / (x1 * x2),
        }[expr].astype(np.float32)
    fin = np.isfinite(want)
    X = np.stack([a, b])[:, fin]
    out, complete = eval_tree_array(tree, X, opts)
    assert complete
    got, exp = _bits(out), _bits(want[fin])
    bad = np.flatnonzero(got != exp)
    assert bad.size == 0, (expr, bad[:5], X[:, bad[:5]].T, out[bad[:5]], want[fin][bad[:5]])


def test_division_special_operands_complete_flags():
    """Zeros, infinities, NaN and subnormals take the full path: flags as IEEE division gives them."""
    opts = Options(binary_operators=["+", "-", "*", "/"], unary_operators=[])
    tree = parse_expression("x1 / x2", opts)
    f32 = np.float32
    cases = [(1.0, 0.0), (0.0, 0.0), (-0.0, 3.0), (5.0, np.inf), (np.inf, 2.0), (np.nan, 1.0),
             (1.0, 1e-45), (1e-45, 1e30), (3e38, 1e-3), (-2.0, -0.0)]
    for x, y in cases:
        base = np.full(1024, 1.5, dtype=np.float32)
        X = np.stack([base, base]).copy()
        X[0, 5], X[1, 5] = f32(x), f32(y)
        out, complete = eval_tree_array(tree, X, opts)
        with np.errstate(all="ignore"):
            q = (X[0] / X[1]).astype(np.float32)
        assert complete == bool(np.isfinite(np.sum(q, dtype=np.float32))), (x, y)
        if complete:
            assert np.array_equal(_bits(out), _bits(q)), (x, y)


def test_exp_fast_path_matches_full_path():
    rng = np.random.default_rng(5)
    m = 4096
    v = rng.uniform(-88.0, 70.0, m).astype(np.float32)
    v[:16] = [88.0, -88.0, 0.0, -0.0, 1e-30, -1e-30, 86.5, -87.99999, 0.5, -0.5, 1.0, 2.0,
              np.float32(np.log(2.0)), 80.0, -80.0, 1e-8]
    forced = v.copy()
    forced[::256] = np.float32(-95.0)  # one row per tile beyond |x| = 88: that tile takes the full path
    opts = Options(binary_operators=["+"], unary_operators=["exp"])
    tree = parse_expression("exp(x1)", opts)
    # exp values up to e^88 ~ 1.65e38: two halves so that no array sum overflows
    for lo, hi in ((0, m // 2), (m // 2, m)):
        fast, c1 = eval_tree_array(tree, v[None, lo:hi], opts)
        full, c2 = eval_tree_array(tree, forced[None, lo:hi], opts)
        assert c1 and c2
        keep = np.ones(hi - lo, dtype=bool)
        keep[(np.arange(lo, hi) % 256) == 0] = False
        assert np.array_equal(_bits(fast)[keep], _bits(full)[keep])


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
@pytest.mark.parametrize("batching", [False, True])
def test_derived_columns_change_nothing(dtype, batching):
    """unary(feature) nodes from the call's derived columns (LOAD_DERIVED) give the same losses and
    flags, bit for bit, as evaluating them in every tree; including columns with Inf / NaN rows
    (exp overflow, log of negatives) and a gathered (minibatch) view."""
    import sr_amd
    from sr_amd import Dataset, eval_loss_batch, flatten_trees, gen_random_population
    from sr_amd.dataset import SubDataset

    rng = np.random.default_rng(11)
    n = 1 << 16
    X = rng.standard_normal((5, n)).astype(dtype)
    X[2, ::97] = dtype(95.0)   # exp(95) overflows f32: derived column with Inf rows
    X[4, ::89] = dtype(-3.0)   # safe_log of a negative: NaN rows
    y = (2 * np.cos(X[3]) + X[0] ** 2 - 2).astype(dtype)
    ds = Dataset(X, y)
    opts = Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp", "log", "sin", "sqrt"])
    tb = flatten_trees(gen_random_population(3000, opts, 5, seed=4), dtype)
    view = SubDataset(ds, rng.integers(0, n, n // 2)) if batching else ds
    ctx = sr_amd.get_context()
    try:
        ctx.set_tuning("derived", 1)
        l1, c1 = eval_loss_batch(tb, view, opts)
        used = ctx.last_derived_columns()
        ctx.set_tuning("derived", 0)
        l0, c0 = eval_loss_batch(tb, view, opts)
        assert ctx.last_derived_columns() == 0
    finally:
        ctx.set_tuning("derived", 1)
    assert used >= 10, used
    assert np.array_equal(c1, c0)
    assert 0.1 < c1.mean() < 0.9
    assert np.array_equal(np.asarray(l1)[c1].view(np.uint64 if dtype == np.float64 else np.uint32),
                          np.asarray(l0)[c0].view(np.uint64 if dtype == np.float64 else np.uint32))


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_probe_modes_change_nothing(dtype):
    """The LDS program cache off, on, or on for the classic launches too, and the dead-tree probe, which only sets hints: with no probe, the first-rows probe, the stress-row probe
    (extreme and nearest-zero rows of each feature, through the gather build and derived columns
    computed over those rows) and a probe before every chunk, losses and flags are identical bit for
    bit.  The data holds rare overflow rows past the first tiles, so the stress rows find trees the
    first rows do not."""
    import sr_amd
    from sr_amd import Dataset, eval_loss_batch, flatten_trees, gen_random_population

    rng = np.random.default_rng(12)
    n = 1 << 18
    X = rng.standard_normal((5, n)).astype(dtype)
    X[1, 200_001] = dtype(95.0)   # exp overflows on one row far from the first tiles
    X[3, 150_003] = dtype(0.0)    # division by zero on one row
    y = (2 * np.cos(X[3]) + X[0] ** 2 - 2).astype(dtype)
    ds = Dataset(X, y)
    opts = Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp", "log"])
    tb = flatten_trees(gen_random_population(4000, opts, 5, seed=6), dtype)
    ctx = sr_amd.get_context()
    res = []
    try:
        for probe, stress, cache in ((0, 0, 1), (2, 0, 1), (2, 1, 1), (1, 1, 1), (2, 1, 0)):
            ctx.set_tuning("probe", probe)
            ctx.set_tuning("stress_probe", stress)
            ctx.set_tuning("code_cache", cache)
            res.append(eval_loss_batch(tb, ds, opts))
    finally:
        ctx.set_tuning("probe", 2)
        ctx.set_tuning("stress_probe", 1)
        ctx.set_tuning("code_cache", 1)
    l0, c0 = res[0]
    assert 0.1 < c0.mean() < 0.9
    u = np.uint64 if dtype == np.float64 else np.uint32
    for l1, c1 in res[1:]:
        assert np.array_equal(c1, c0)
        assert np.array_equal(np.asarray(l1)[c1].view(u), np.asarray(l0)[c0].view(u))


@pytest.mark.parametrize("dtype,n_rows,n_trees", [(np.float32, 100_000, 31), (np.float64, 100, 40), (np.float32, 3000, 300)])
def test_small_call_latency_options_change_nothing(dtype, n_rows, n_trees):
    """The search's call shapes under the latency options: results written by the kernel into pinned
    host memory ("host_io"), the partial reduction in the launch ("fused_reduce"), in a separate launch
    or on the host from partials the kernel wrote into pinned memory ("host_reduce"): losses and flags
    bit for bit equal — with the in-order fold ("ref_fold" 1, the default, which keeps the partials on
    the device) and with the f64 sums ("ref_fold" 0)."""
    import sr_amd
    from sr_amd import Dataset, eval_loss_batch, flatten_trees, gen_random_population

    rng = np.random.default_rng(31)
    X = rng.uniform(0.5, 2.0, (5, n_rows)).astype(dtype)
    y = (X[0] * X[1] * X[2] / (X[3] * X[4] ** 2 + 1)).astype(dtype)
    ds = Dataset(X, y)
    opts = Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp"])
    tb = flatten_trees(gen_random_population(n_trees, opts, 5, max_size=20, seed=31), dtype)
    ctx = sr_amd.get_context()
    for ref_fold in (1, 0):
        res = []
        try:
            ctx.set_tuning("ref_fold", ref_fold)
            for host_io, fused, hred in ((1, 1 << 30, 0), (1, 0, 0), (0, 0, 0), (1, 0, 1 << 20), (0, 0, 1 << 20)):
                ctx.set_tuning("host_io", host_io)
                ctx.set_tuning("fused_reduce", fused)
                ctx.set_tuning("host_reduce", hred)
                res.append(eval_loss_batch(tb, ds, opts))
        finally:
            ctx.set_tuning("ref_fold", 1)
            ctx.set_tuning("host_io", 1)
            ctx.set_tuning("fused_reduce", 0)
            ctx.set_tuning("host_reduce", 8192)
        l0, c0 = res[0]
        assert c0.mean() > 0.2
        for l1, c1 in res[1:]:
            assert np.array_equal(c1, c0)
            assert np.array_equal(np.asarray(l1).view(np.uint8), np.asarray(l0).view(np.uint8)), ref_fold
