"""GPU parity: libsr_amd (HIP, through the C ABI) vs the CPU oracle and the reference's known answers.

Bars (BASELINE.json north_star): per-tree `complete` flags bit-exact; losses within 1e-4 relative
(f32) / 1e-10 relative (f64) of the oracle; predictions within the reference tests' tolerances.
"""
import ctypes

import numpy as np
import pytest

import sr_amd
from oracle import Oracle
from sr_amd import (Dataset, Node, Options, batch, eval_loss, eval_loss_batch, eval_tree_array, eval_tree_array_batch,
                    flatten_trees, gen_random_population, parse_expression)
from sr_amd import _lib
from parity_util import PERTURB_SEEDS, assert_losses_within, loss_tolerance


pytestmark = pytest.mark.gpu

C2_OPTS = dict(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp", "log"])
FULL_OPTS = dict(
    binary_operators=["+", "-", "*", "/", "^", "max", "min", "mod", ">", "<", "cond", "logical_or"],
    unary_operators=["cos", "exp", "log", "sin", "tan", "sqrt", "abs", "tanh", "neg", "square", "cube",
                     "log1p", "atan", "asinh", "relu", "inv", "erf", "sign", "floor"],
)


def _dt(name):
    return np.float32 if name == "float32" else np.float64


def _c2_data(n, nf=5, dtype=np.float32, seed=2):
    rng = np.random.default_rng(seed)
    X = rng.standard_normal((nf, n)).astype(dtype)
    y = (2 * np.cos(X[3].astype(np.float64)) + X[0].astype(np.float64) ** 2 - 2
         + 0.1 * np.random.default_rng(seed + 1).standard_normal(n)).astype(dtype)
    return X, y


def _rel(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    both_inf = np.isinf(a) & np.isinf(b) & (np.sign(a) == np.sign(b))
    with np.errstate(invalid="ignore"):
        return np.where(both_inf, 0.0, np.abs(a - b) / np.maximum(np.abs(b), 1e-30))


# ------------------------------------------------------------------ reference known answers
def test_golden_fused_shapes(golden):
    g = golden["fused_shapes"]
    opts = Options(binary_operators=g["binary_operators"], unary_operators=g["unary_operators"])
    X = np.array(g["X"], dtype=np.float32)
    trees = [parse_expression(c["expr"], opts) for c in g["cases"]]
    out, comp = eval_tree_array_batch(trees, Dataset(X), opts)
    for k, case in enumerate(g["cases"]):
        assert comp[k], case["expr"]
        err = np.abs(out[k].astype(np.float64) - np.array(case["expected"])) / X.shape[1]
        assert np.all(err < g["tolerance_abs_over_N"]), (case["expr"], err.max())


def test_golden_nan_detection(golden):
    g = golden["nan_detection"]
    opts = Options(binary_operators=g["binary_operators"], unary_operators=g["unary_operators"])
    for case in g["cases"]:
        dt = _dt(case["dtype"])
        t = parse_expression(case["expr"], opts)
        X = np.array(case["X"], dtype=dt)
        _, complete = eval_tree_array(t, X, opts)
        assert complete is g["expected_complete"], case
        d = Dataset(X, np.zeros(X.shape[1], dtype=dt))
        loss, comp = eval_loss_batch([t], d, opts)
        assert not comp[0] and np.isinf(loss[0]), case


def test_golden_batched_dataset_mse(golden):
    g = golden["batched_mse"]
    opts = Options(binary_operators=g["binary_operators"], unary_operators=g["unary_operators"])
    d = Dataset(np.array(g["X"]), np.array(g["y"]))
    t = parse_expression(g["expr"], opts)
    for case in g["cases"]:
        view = d if case["indices"] is None else batch(d, case["indices"])
        assert eval_loss(t, view, opts) == pytest.approx(case["loss"], rel=1e-12)


@pytest.mark.parametrize("loss_name", ["L1DistLoss", "L2DistLoss"])
def test_golden_losses(golden, loss_name):
    g = golden["losses"]
    x = np.array(g["x"], dtype=np.float32)
    y = np.array(g["y"], dtype=np.float32)
    w = np.array(g["w"], dtype=np.float32)
    opts = Options(binary_operators=["+"], unary_operators=[], elementwise_loss=loss_name)
    t = parse_expression("x1", opts)
    assert abs(float(eval_loss(t, Dataset(x[None, :], y), opts)) - g[loss_name]["mean"]) < g["tolerance"]
    assert abs(float(eval_loss(t, Dataset(x[None, :], y, weights=w), opts)) - g[loss_name]["weighted"]) < g["tolerance"]


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_golden_safe_operators(golden, dtype):
    g = golden["safe_operators"]
    for case in g["unary"]:
        opts = Options(binary_operators=["+"], unary_operators=[case["op"]])
        out, _ = eval_tree_array(parse_expression(f"{case['op']}(x1)", opts), np.array([[case["x"]]], dtype=dtype), opts)
        if case["expected"] == "nan":
            assert np.isnan(out[0]), case
        else:
            assert abs(float(out[0]) - case["expected"]) < g["tolerance"], case
    for case in g["binary"]:
        opts = Options(binary_operators=[case["op"]], unary_operators=[])
        t = Node(op=1, l=Node(feature=1), r=Node(feature=2))
        out, _ = eval_tree_array(t, np.array([[case["x"]], [case["y"]]], dtype=dtype), opts)
        if case["expected"] == "nan":
            assert np.isnan(out[0]), case
        else:
            assert abs(float(out[0]) - case["expected"]) < g["tolerance"], case


def test_golden_tree_construction(golden):
    g = golden["tree_construction"]
    for case in g["cases"]:
        dt = _dt(case["dtype"])
        una = case["unaop"]
        opts = Options(binary_operators=g["binary_operators"], unary_operators=[una, "abs"],
                       parsimony=g["parsimony_default"])
        good = parse_expression(g["good_expr"].replace("UNAOP", una), opts)
        bad = parse_expression(g["bad_expr"].replace("UNAOP", una), opts)
        d = Dataset(np.array(case["X"], dtype=dt), np.array(case["y"], dtype=dt))
        l = eval_loss(good, d, opts)
        assert abs(float(l)) < case["tolerance"], (una, case["dtype"], float(l))
        assert l == sr_amd.eval_cost(d, good, opts)[1]
        assert sr_amd.eval_cost(d, good, opts)[0] < sr_amd.eval_cost(d, bad, opts)[0]


# ------------------------------------------------------------------ random populations vs oracle
@pytest.mark.parametrize("opts_kw,n,n_trees,seed", [
    (C2_OPTS, 4096, 3000, 1),
    (C2_OPTS, 5000, 1500, 7),      # ragged rows (not a multiple of the 1024-row tile)
    (FULL_OPTS, 3000, 2000, 3),
    (C2_OPTS, 97, 500, 11),        # fewer rows than one wave
])
def test_population_f32_vs_oracle(opts_kw, n, n_trees, seed):
    opts = Options(**opts_kw)
    X, y = _c2_data(n, seed=seed)
    trees = gen_random_population(n_trees, opts, 5, max_size=30, seed=seed)
    tb = flatten_trees(trees, np.float32)
    loss, comp = eval_loss_batch(tb, Dataset(X, y), opts)
    orc = Oracle.from_options(opts)
    tol, o_loss, o_comp, n_wide = loss_tolerance(orc, tb, X, y)
    mism = np.nonzero(comp != o_comp)[0]
    assert len(mism) == 0, [(int(k), sr_amd.string_tree(tb.tree(int(k)), opts.operators)) for k in mism[:5]]
    assert np.all(np.isinf(loss[~comp]))
    # every complete tree, no exclusions: the 1e-4 bar, or 4x the tree's own libm spread
    assert_losses_within(loss, o_loss, comp, tol)
    assert n_wide < 0.2 * comp.sum()
    assert np.median(_rel(loss[comp], o_loss[comp])) < 1e-6
    # against the reference-order accumulation (sequential f32 fold) too
    ref_loss, _ = orc.eval_loss_batch(tb, X, y, accum="ref", n_threads=8)
    assert_losses_within(loss, ref_loss, comp, np.maximum(tol, 1e-4 * np.abs(ref_loss.astype(np.float64))))


def test_population_f64_vs_oracle():
    opts = Options(**C2_OPTS)
    X, y = _c2_data(3000, dtype=np.float64, seed=5)
    trees = gen_random_population(1500, opts, 5, max_size=30, dtype=np.float64, seed=5)
    tb = flatten_trees(trees, np.float64)
    loss, comp = eval_loss_batch(tb, Dataset(X, y), opts)
    orc = Oracle.from_options(opts)
    # north_star's Float64 bar, per tree and for EVERY complete tree: 1e-10 relative, or 4x the tree's
    # own spread under +-1-ulp libm perturbations (the same rule as Float32's 1e-4)
    tol, o_loss, o_comp, n_wide = loss_tolerance(orc, tb, X, y, rel_bar=1e-10)
    assert np.array_equal(comp, o_comp)
    assert_losses_within(loss, o_loss, comp, tol, "f64")
    assert n_wide < 0.2 * comp.sum()
    assert np.median(_rel(loss[comp], o_loss[comp])) < 1e-13


@pytest.mark.parametrize("dtype,builds", [(np.float32, (0, 16, 8)), (np.float64, (0, 8, 4))])
def test_kernel_builds_and_launch_orders_agree(dtype, builds):
    """Every interpreter build a call can pick (register-stack or LDS-stack operand stack, rows per
    lane) and both launch orders (cost ranks dealt over tree groups, or contiguous) against the oracle;
    one build's results are bit-identical whatever the launch order."""
    opts = Options(**C2_OPTS)
    X, y = _c2_data(20000, dtype=dtype, seed=17)
    tb = flatten_trees(gen_random_population(1200, opts, 5, max_size=30, dtype=dtype, seed=17), dtype)
    d = Dataset(X, y)
    orc = Oracle.from_options(opts)
    rel_bar = 1e-10 if dtype == np.float64 else 1e-4
    tol, o_loss, o_comp, _ = loss_tolerance(orc, tb, X, y, rel_bar=rel_bar)
    ctx = sr_amd.get_context()
    try:
        for rpl in builds:
            ctx.set_tuning("rows_per_lane", rpl)
            runs = []
            for bal in (1, 0):
                ctx.set_tuning("balance", bal)
                loss, comp = eval_loss_batch(tb, d, opts)
                assert np.array_equal(comp, o_comp), (rpl, bal)
                assert_losses_within(loss, o_loss, comp, tol, f"rows_per_lane={rpl} balance={bal}")
                runs.append(loss)
            assert np.array_equal(runs[0], runs[1]), rpl
    finally:
        ctx.set_tuning("rows_per_lane", 0)
        ctx.set_tuning("balance", 1)


def test_predictions_vs_oracle():
    opts = Options(**FULL_OPTS)
    X, _ = _c2_data(777, seed=9)
    trees = gen_random_population(300, opts, 5, seed=9)
    tb = flatten_trees(trees, np.float32)
    out, comp = eval_tree_array_batch(tb, Dataset(X), opts)
    orc = Oracle.from_options(opts)
    compared = total = 0
    for k in range(tb.n_trees):
        o, c = orc.eval_tree_array(tb, k, X)
        assert comp[k] == c, (k, sr_amd.string_tree(tb.tree(k), opts.operators))
        if c:
            # every row: 1e-4 relative (1e-6 absolute near zero), or 4x the row's own spread under
            # +-1-ulp libm perturbations (cancellation, or a floor/sign/comparison sitting on its
            # threshold, amplifies last-bit libm differences)
            o64 = o.astype(np.float64)
            spread = np.zeros(o.shape)
            for seed in PERTURB_SEEDS:
                p, _ = orc.eval_tree_array(tb, k, X, perturb=seed)
                with np.errstate(invalid="ignore"):
                    d = np.abs(p.astype(np.float64) - o64)
                spread = np.maximum(spread, np.where(np.isfinite(d), d, np.inf))
            tol = np.maximum(1e-4 * np.abs(o64) + 1e-6, 4 * spread)
            dev = out[k].astype(np.float64)
            same_nonfinite = (~np.isfinite(dev)) & (~np.isfinite(o64)) & ((dev == o64) | (np.isnan(dev) & np.isnan(o64)))
            with np.errstate(invalid="ignore"):
                ok = same_nonfinite | (np.abs(dev - o64) <= tol)
            compared += int(np.sum(spread <= 2e-5 * np.maximum(np.abs(o64), 1e-3)))
            total += o.size
            assert ok.all(), (k, sr_amd.string_tree(tb.tree(k), opts.operators), np.nonzero(~ok)[0][:5])
    assert compared > 0.8 * total  # most rows of complete trees are well-conditioned (plain bar)


def test_weighted_and_gather_vs_oracle():
    opts = Options(**C2_OPTS)
    X, y = _c2_data(6000, seed=13)
    w = np.abs(np.random.default_rng(14).standard_normal(6000)).astype(np.float32) + 0.1
    d = Dataset(X, y, weights=w)
    trees = gen_random_population(800, opts, 5, seed=13)
    tb = flatten_trees(trees, np.float32)
    orc = Oracle.from_options(opts)
    loss, comp = eval_loss_batch(tb, d, opts)
    tol, ol, oc, _ = loss_tolerance(orc, tb, X, y, w=w)
    assert np.array_equal(comp, oc)
    assert_losses_within(loss, ol, comp, tol)
    # SubDataset (minibatch with replacement): gather path
    idx = np.random.default_rng(15).integers(0, 6000, size=1500)
    sub = batch(d, idx)
    loss, comp = eval_loss_batch(tb, sub, opts)
    tol, ol, oc, _ = loss_tolerance(orc, tb, X[:, idx], y[idx], w=w[idx])
    assert np.array_equal(comp, oc)
    assert_losses_within(loss, ol, comp, tol)


def test_l1_loss_vs_oracle():
    opts = Options(**C2_OPTS, elementwise_loss="L1DistLoss")
    X, y = _c2_data(2048, seed=21)
    tb = flatten_trees(gen_random_population(600, opts, 5, seed=21), np.float32)
    loss, comp = eval_loss_batch(tb, Dataset(X, y), opts)
    tol, ol, oc, _ = loss_tolerance(Oracle.from_options(opts), tb, X, y, loss_kind=1)
    assert np.array_equal(comp, oc)
    assert_losses_within(loss, ol, comp, tol)


# ------------------------------------------------------------------ edge cases
def test_edge_trees():
    opts = Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp", "log"])
    X, y = _c2_data(3000, seed=31)
    X[2, 17] = 1e30  # one huge value in feature 3
    exprs = [
        "x1", "2.5", "inf", "nan", "cos(3.0)", "cos(inf)", "exp(1000.0)", "x1 + inf", "x1 * nan",
        "exp(x1 * 100.0)", "log(x2)", "log(0.0 * x1)", "x3 * 1e10", "x3 * x3",
        "cos(x1 / 0.0)", "exp(cos(x1 * x2))", "(x1 + x2) * (x3 - x4)", "((x1 * x2) + (x3 * x4)) * ((x5 + x1) - (x2 * x3))",
        "1e36 * 1.0", "x1 * 0.0 + 1e34", "exp(88.0 + x1 * 0.0)", "exp(89.0 + x1 * 0.0)",
        "exp(-200.0 * x1)", "1.0 / (x1 - x1)", "(x1 - x1) / (x2 - x2)",
    ]
    trees = [parse_expression(e, opts) for e in exprs]
    tb = flatten_trees(trees, np.float32)
    loss, comp = eval_loss_batch(tb, Dataset(X, y), opts)
    ol, oc = Oracle.from_options(opts).eval_loss_batch(tb, X, y, accum="f64")
    for k, e in enumerate(exprs):
        assert comp[k] == oc[k], (e, comp[k], oc[k])
        if oc[k]:
            assert _rel(loss[k], ol[k]) < 1e-4 or (np.isinf(loss[k]) and np.isinf(ol[k])), (e, loss[k], ol[k])


def test_sum_overflow_exact_path():
    """Values finite row by row but whose array sum overflows Float32: DE's isfinite(sum(x)) check
    flags them; values just below the limit must stay complete (exact-sum path)."""
    opts = Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos"])
    n = 4000
    X = np.ones((1, n), dtype=np.float32)
    y = np.zeros(n, dtype=np.float32)
    exprs = [
        "x1 * 1e35",          # 4000 * 1e35 = 4e38 > FLT_MAX -> incomplete
        "x1 * 5e34",          # 2e38 -> complete (the root check passes; loss itself overflows to Inf)
        "cos(x1 * 1e35)",     # fused: child of cos is not array-checked; cos bounded -> complete
        "cos(x1) * 1e35",     # 4000 * 0.54e35 = 2.16e38 -> complete
        "cos(x1 * 0.0) * 1e35 + x1 * 0.0",  # 4e38 at a checked node -> incomplete
    ]
    trees = [parse_expression(e, opts) for e in exprs]
    tb = flatten_trees(trees, np.float32)
    _, comp = eval_loss_batch(tb, Dataset(X, y), opts)
    _, oc = Oracle.from_options(opts).eval_loss_batch(tb, X, y)
    assert list(comp) == list(oc), list(zip(exprs, comp, oc))
    assert list(oc) == [False, True, True, True, False]


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_untracked_outputs_keep_the_checks(dtype):
    """SR_TRACK_LITE (sr_tile_impl.h): + and - of stack values / features and cos, sin, neg, abs, sqrt
    leave the deferred checks' running max; the launch's thresholds are divided by the largest tree's
    node count, and data at or above that bound tracks + and - again.  Positive data at scales around
    those bounds (including sums of untracked nodes whose array sums overflow): flags equal the
    oracle's, losses within the per-tree bar."""
    opts = Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "sin", "sqrt", "abs", "neg"])
    n = 4000
    fmax = float(np.finfo(dtype).max)
    tbig = fmax / (2 * n)
    exprs = ["((x1 + x2) + x3) + x4", "(x1 + x2) - (x3 + x4)",
             "((x1 + x2) + (x3 + x4)) + ((x5 + x1) + (x2 + x3))", "sqrt(abs((x1 + x2) + x3))",
             "neg((x1 + x2) + (x3 + x4))", "cos(x1 + x2) + x3", "sin(x1 - x2) * x3", "(x1 + x2) * 2.0",
             "x1 * 3.0 + x2", "((x1 + x2) + x3) / 0.5", "x1 + x2", "abs(x1 - x2) + cos(x3)"]
    trees = [parse_expression(e, opts) for e in exprs]
    tb = flatten_trees(trees, dtype)
    orc = Oracle.from_options(opts)
    rng = np.random.default_rng(5)
    # below tbig / L, between tbig / L and tbig (track_x), past the point where 4-leaf sums overflow
    for scale in (1e-3 * tbig, 0.02 * tbig, 0.3 * tbig, 0.52 * tbig, 2.2 * tbig / 2, 1e4):
        X = (scale * (1.0 + 0.01 * rng.random((5, n)))).astype(dtype)
        y = np.zeros(n, dtype=dtype)
        loss, comp = eval_loss_batch(tb, Dataset(X, y), opts)
        tol, ol, oc, _ = loss_tolerance(orc, tb, X, y)
        assert np.array_equal(comp, oc), (scale, [(e, c, o) for e, c, o in zip(exprs, comp, oc) if c != o])
        assert_losses_within(loss, ol, comp, tol, scale)


def test_ragged_sizes_and_determinism():
    opts = Options(**C2_OPTS)
    trees = gen_random_population(400, opts, 5, seed=41)
    tb = flatten_trees(trees, np.float32)
    orc = Oracle.from_options(opts)
    for n in (1, 2, 63, 64, 255, 1023, 1024, 1025, 4097):
        X, y = _c2_data(n, seed=n)
        d = Dataset(X, y)
        l1, c1 = eval_loss_batch(tb, d, opts)
        l2, c2 = eval_loss_batch(tb, d, opts)
        assert np.array_equal(l1, l2) and np.array_equal(c1, c2)  # bit-reproducible
        tol, ol, oc, _ = loss_tolerance(orc, tb, X, y)
        assert np.array_equal(c1, oc), n
        assert_losses_within(l1, ol, c1, tol, n)


def test_chunked_batch_matches_pieces(monkeypatch):
    """With SR_AMD_CHUNKS, >= 4096 trees are compiled and launched in chunks (the host compiles chunk
    c+1 while the device runs chunk c): per-tree results must not depend on the chunking —
    bit-identical to evaluating each piece alone — and an error names the tree's index in the whole
    batch."""
    monkeypatch.setenv("SR_AMD_CHUNKS", "4")
    ctx = sr_amd.device.DeviceContext(0)  # reads the environment at creation
    opts = Options(**C2_OPTS)
    X, y = _c2_data(3000, seed=71)
    d = Dataset(X, y)
    trees = gen_random_population(9000, opts, 5, max_size=30, seed=71)
    loss, comp = eval_loss_batch(flatten_trees(trees, np.float32), d, opts, ctx=ctx)
    parts = [eval_loss_batch(flatten_trees(trees[i:i + 1500], np.float32), d, opts, ctx=ctx) for i in range(0, 9000, 1500)]
    assert np.array_equal(comp, np.concatenate([p[1] for p in parts]))
    assert np.array_equal(loss, np.concatenate([p[0] for p in parts]))
    sub = flatten_trees(trees[6500:7300], np.float32)  # straddles a chunk boundary
    tol, ol, oc, _ = loss_tolerance(Oracle.from_options(opts), sub, X, y)
    assert np.array_equal(comp[6500:7300], oc)
    assert_losses_within(loss[6500:7300], ol, oc, tol)
    bad = list(trees)
    bad[8500] = Node(feature=9)  # feature out of range, in the last chunk
    with pytest.raises(sr_amd.SRError, match="tree 8500"):
        eval_loss_batch(bad, d, opts, ctx=ctx)
    l2, c2 = eval_loss_batch(flatten_trees(trees, np.float32), d, opts, ctx=ctx)  # the context still works
    assert np.array_equal(l2, loss)
    d.free_device()
    ctx.close()
    # the default context: two chunks (a small first one while the rest compiles)
    d2 = Dataset(X, y)
    l3, c3 = eval_loss_batch(flatten_trees(trees, np.float32), d2, opts)
    assert np.array_equal(l3, loss) and np.array_equal(c3, comp)


@pytest.mark.parametrize("mode", ["0", "1"])
def test_dead_tree_probe_is_invisible(monkeypatch, mode):
    """The dead-tree probe launch (first 4 row tiles, hints only; SR_AMD_PROBE: 0 off, 1 every
    chunk, 2 = default, the chunks after the first) changes no result: contexts in every mode give
    bit-identical losses and flags, and all equal the oracle's flags.  6600 trees -> two chunks."""
    opts = Options(**C2_OPTS)
    X, y = _c2_data(40000, seed=81)
    tb = flatten_trees(gen_random_population(6600, opts, 5, max_size=30, seed=81), np.float32)
    loss, comp = eval_loss_batch(tb, Dataset(X, y), opts)
    assert sr_amd.device.get_context().last_launches() == 2
    monkeypatch.setenv("SR_AMD_PROBE", mode)
    ctx = sr_amd.device.DeviceContext(0)
    d2 = Dataset(X, y)
    l2, c2 = eval_loss_batch(tb, d2, opts, ctx=ctx)
    d2.free_device()
    ctx.close()
    assert np.array_equal(comp, c2) and np.array_equal(loss, l2)
    _, oc = Oracle.from_options(opts).eval_loss_batch(tb, X, y, n_threads=8)
    assert np.array_equal(comp, oc)
    assert 0.2 < comp.mean() < 0.8  # the population has plenty of dead trees for the probe


def test_empty_batch_and_errors():
    opts = Options(**C2_OPTS)
    X, y = _c2_data(100)
    d = Dataset(X, y)
    loss, comp = eval_loss_batch([], d, opts)
    assert loss.shape == (0,)
    bad = Node(feature=9)  # feature out of range
    with pytest.raises(sr_amd.SRError):
        eval_loss_batch([bad], d, opts)
    with pytest.raises(IndexError):
        batch(d, [0, 100])


# ------------------------------------------------------------------ large sizes: size-independent properties
def test_large_rows_properties():
    """1M rows (BASELINE C2 size): linear trees against LossFunctions' in-order Float32 fold of their
    Float32 predictions (numpy's add.accumulate is a sequential fold), bit for bit; the f64 closed form
    is ~1e-3 away at this size (the fold's own rounding)."""
    opts = Options(**C2_OPTS)
    n = 1 << 20
    X, y = _c2_data(n, seed=51)
    d = Dataset(X, y)
    exprs = ["x1", "x1 * 2.0", "x1 + x2", "cos(x4) * 2.0 + x1 * x1 - 2.0"]
    trees = [parse_expression(e, opts) for e in exprs]
    loss, comp = eval_loss_batch(trees, d, opts)
    assert comp.all()
    pred = [X[0], X[0] * np.float32(2.0), X[0] + X[1]]
    for k in range(3):
        d2 = ((pred[k] - y) * (pred[k] - y)).astype(np.float32)
        fold = np.float32(np.add.accumulate(d2, dtype=np.float32)[-1] / np.float32(n))
        assert loss[k].view(np.uint32) == fold.view(np.uint32), (exprs[k], loss[k], fold)
        exact = np.mean((pred[k].astype(np.float64) - y) ** 2)
        assert _rel(loss[k], exact) < 1e-2
    # the generating formula: loss ~ noise variance 0.01
    assert abs(float(loss[3]) - 0.01) < 1e-3
    # same answer through a SubDataset covering all rows in order (gather path): bit for bit
    l2, c2 = eval_loss_batch(trees, batch(d, np.arange(n)), opts)
    assert np.array_equal(l2.view(np.uint32), loss.view(np.uint32))


def test_row_sharded_partials_match_single():
    """The multi-GPU building block: Σ over row shards of sr_eval_loss_partials (f64 partial sums) == one
    full eval with the f64 sums ("ref_fold" 0)."""
    opts = Options(**C2_OPTS)
    n = 20000
    X, y = _c2_data(n, seed=61)
    tb = flatten_trees(gen_random_population(700, opts, 5, seed=61), np.float32)
    ctx = sr_amd.get_context()
    ctx.set_tuning("ref_fold", 0)
    try:
        full_loss, full_comp = eval_loss_batch(tb, Dataset(X, y), opts)
    finally:
        ctx.set_tuning("ref_fold", 1)
    oid = ctx.opset_id(opts.operators)
    sums = np.zeros(tb.n_trees)
    flags = np.zeros(tb.n_trees, dtype=np.uint32)
    shards = [Dataset(np.ascontiguousarray(X[:, a:b]), np.ascontiguousarray(y[a:b])) for a, b in ((0, 7000), (7000, n))]
    s = tb.to_struct()
    for sh in shards:
        ps = np.zeros(tb.n_trees)
        pf = np.zeros(tb.n_trees, dtype=np.uint32)
        _lib.check(_lib.lib.sr_eval_loss_partials(ctx.handle, sh.device_handle(ctx), oid, ctypes.byref(s), n, 0,
                                                  ps.ctypes.data_as(ctypes.c_void_p), pf.ctypes.data_as(ctypes.c_void_p), 0))
        sums += ps
        flags |= pf
    out = np.empty(tb.n_trees, dtype=np.float32)
    comp = np.empty(tb.n_trees, dtype=np.uint8)
    _lib.check(_lib.lib.sr_finalize_losses(_lib.SR_DTYPE_F32, tb.n_trees, sums.ctypes.data_as(ctypes.c_void_p),
                                           flags.ctypes.data_as(ctypes.c_void_p), float(n), None, 0, None,
                                           out.ctypes.data_as(ctypes.c_void_p), comp.ctypes.data_as(ctypes.c_void_p)))
    assert np.array_equal(comp.astype(bool), full_comp)
    assert np.max(_rel(out[full_comp], full_loss[full_comp])) < 1e-6


@pytest.mark.parametrize("max_rb", [1, 7, 1000])
def test_row_block_bound_keeps_results(monkeypatch, max_rb):
    """SR_AMD_MAX_ROW_BLOCKS only regroups rows into workgroups (one tile per block up to every tile
    in one block): flags and losses (the in-order fold) stay bit-identical to the default grid, and
    equal the oracle's."""
    opts = Options(**C2_OPTS)
    X, y = _c2_data(100_000, seed=83)
    trees = flatten_trees(gen_random_population(1500, opts, 5, max_size=30, seed=83), np.float32)
    d = Dataset(X, y)
    ref_loss, ref_comp = eval_loss_batch(trees, d, opts)
    monkeypatch.setenv("SR_AMD_MAX_ROW_BLOCKS", str(max_rb))
    ctx = sr_amd.device.DeviceContext(0)  # reads the environment at creation
    d2 = Dataset(X, y)  # a device dataset belongs to one context
    loss, comp = eval_loss_batch(trees, d2, opts, ctx=ctx)
    assert np.array_equal(comp, ref_comp)
    fin = np.isfinite(ref_loss)
    assert np.array_equal(fin, np.isfinite(loss))
    # the in-order fold does not depend on how rows are grouped: bit for bit
    assert np.array_equal(loss[fin].view(np.uint32), ref_loss[fin].view(np.uint32))
    sub = flatten_trees([trees.tree(i) for i in range(0, 1500, 15)], np.float32)
    tol, ol, oc, _ = loss_tolerance(Oracle.from_options(opts), sub, X, y)
    assert np.array_equal(comp[::15], oc)
    assert_losses_within(loss[::15], ol, oc, tol)
    d2.free_device()
    d.free_device()
    ctx.close()


# ------------------------------------------------------------------ exact validity path (Julia order)
def _adversarial_columns():
    """Checked arrays on which an exact (f64) sum and Julia's T-precision pairwise sum disagree
    (tests/test_jsum.py pins the verdicts on the CPU)."""
    from test_jsum import cases

    return {k: v for k, v in cases().items() if k not in ("one", "fifteen")}


@pytest.mark.parametrize("name", list(_adversarial_columns()))
def test_exact_path_follows_julia_sum_order(name):
    """Flags of trees whose checked arrays are the adversarial columns: the device (deferred checks
    -> BIG -> EXACT pass) must agree with the oracle's isfinite(Julia sum) bit for bit."""
    col = _adversarial_columns()[name]
    n = len(col)
    X = np.stack([col, np.zeros(n, np.float32), np.ones(n, np.float32)]).astype(np.float32)
    y = np.zeros(n, dtype=np.float32)
    opts = Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos"])
    exprs = ["x1 * 1.0", "(x1 * 1.0) + (x2 * 0.0)", "cos(x2) * (x1 * x3)", "(x1 - x2) / (x3 * 1.0)", "x1 + x2"]
    tb = flatten_trees([parse_expression(e, opts) for e in exprs], np.float32)
    _, comp = eval_loss_batch(tb, Dataset(X, y), opts)
    _, oc = Oracle.from_options(opts).eval_loss_batch(tb, X, y, n_threads=4)
    assert list(comp) == list(oc), (name, list(zip(exprs, comp, oc)))


def test_row_sharded_packed_with_exact_path():
    """Two row shards on one GPU through the multi-GPU building blocks — packed partials (one
    all-reduce's worth), Julia-order folds per shard (the boundary falls inside a leaf block),
    sr_jsum_finite, sr_finalize_losses — equal the single-GPU result bit for bit in the flags."""
    from sr_amd.distributed import finalize, gpu_jsum, gpu_max_checks, gpu_partials_packed, jsum_finite, unpack_flags
    from test_jsum import cases

    opts = Options(**C2_OPTS)
    n = 9000
    X, y = _c2_data(n, seed=91)
    X[2] = np.resize(cases()["mixed_overflow_pairwise"], n)  # x3 carries +-2e35 blocks
    X[4, :4000] = 3e38 / 4000 * 1.3                           # x5's array sums just past FLT_MAX
    trees = gen_random_population(600, opts, 5, seed=91)
    trees += [parse_expression(e, opts) for e in ("x3 * 1.0", "x3 + x1", "x5 * 1.0", "(x5 * 0.5) + (x1 * 1.0)")]
    tb = flatten_trees(trees, np.float32)
    ctx = sr_amd.get_context()
    ctx.set_tuning("ref_fold", 0)  # (the building blocks return f64 sums)
    try:
        full_loss, full_comp = eval_loss_batch(tb, Dataset(X, y), opts)
    finally:
        ctx.set_tuning("ref_fold", 1)
    cut = 4321
    shards = [Dataset(np.ascontiguousarray(X[:, :cut]), np.ascontiguousarray(y[:cut])),
              Dataset(np.ascontiguousarray(X[:, cut:]), np.ascontiguousarray(y[cut:]))]
    packed = sum(gpu_partials_packed(tb, sh, opts, n) for sh in shards)
    sums, flags = unpack_flags(packed)
    big = np.nonzero(((flags & (_lib.SR_FLAG_NONFINITE | _lib.SR_FLAG_STATIC)) == 0) & ((flags & _lib.SR_FLAG_BIG) != 0))[0]
    assert big.size >= 2
    mc = gpu_max_checks(tb, opts)
    folds = [gpu_jsum(tb, sh, opts, big, mc, off, n) for sh, off in zip(shards, (0, cut))]
    fin = jsum_finite(np.float32, n, [0, cut, n], [f.reshape(big.size * mc, -1) for f in folds])
    ok = fin.reshape(big.size, mc).all(axis=1)
    loss, comp = finalize(np.float32, sums, flags, float(n), big, ok)
    assert np.array_equal(comp, full_comp)
    assert np.max(_rel(loss[full_comp], full_loss[full_comp]), initial=0.0) < 1e-6
    _, oc = Oracle.from_options(opts).eval_loss_batch(tb, X, y, n_threads=8)
    assert np.array_equal(comp, oc)


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_exact_pass_after_a_probed_launch(dtype):
    """Trees the dead-tree probe already sees BIG over the stress rows (mixed +-2e35 blocks, sums just
    past floatmax) go through the exact-sum pass after the main launch; with a probe before every
    chunk the flags must equal the oracle's and the call must equal the unprobed one.  (Round 5's
    speculative pass that ran this pass during the main launch was measured neutral and removed.)"""
    from test_jsum import cases

    opts = Options(**C2_OPTS)
    n = 1 << 16
    X, y = _c2_data(n, seed=93)
    X, y = X.astype(dtype), y.astype(dtype)
    big = float(np.finfo(dtype).max)
    blocks = np.resize(cases()["mixed_overflow_pairwise"], n).astype(np.float64)  # +-2e35 blocks
    X[2] = (blocks * (big / 3.4028235e38)).astype(dtype)
    X[4, :30000] = big / 30000 * 1.3  # x5's array sums just past floatmax
    trees = gen_random_population(600, opts, 5, seed=93)
    trees += [parse_expression(e, opts) for e in ("x3 * 1.0", "x3 + x1", "x5 * 1.0", "(x5 * 0.5) + (x1 * 1.0)",
                                                  "cos(x3) + (x5 * 1.0)", "(x3 * x2) - x5")]
    tb = flatten_trees(trees, dtype)
    ds = Dataset(X, y)
    ctx = sr_amd.get_context()
    try:
        ctx.set_tuning("probe", 1)  # (a probe before every chunk: this call is below the default's size)
        loss_s, comp_s = eval_loss_batch(tb, ds, opts)
        n_exact = ctx.last_exact_trees()
        ctx.set_tuning("probe", 0)
        loss_o, comp_o = eval_loss_batch(tb, ds, opts)
    finally:
        ctx.set_tuning("probe", 2)
    assert n_exact > 0
    assert np.array_equal(comp_s, comp_o)
    assert np.array_equal(loss_s, loss_o, equal_nan=True)
    _, oc = Oracle.from_options(opts).eval_loss_batch(tb, X, y, n_threads=8)
    assert np.array_equal(comp_s, oc)


def test_wide_f64_dataset_large_view_falls_back_to_classic_kernel():
    """Float64 over >= 2^17 rows defaults to the 8-rows/lane register-stack kernel,
    whose X tile (4096 (nf + 1) bytes) passes 160 KiB at ~40 features; such a call must run the classic
    kernel instead of failing, and agree with the oracle."""
    opts = Options(**C2_OPTS)
    nf, n = 48, 1 << 17
    rng = np.random.default_rng(44)
    X = rng.standard_normal((nf, n))
    y = np.cos(X[3]) + X[40] ** 2
    tb = flatten_trees(gen_random_population(200, opts, nf, max_size=20, dtype=np.float64, seed=44), np.float64)
    loss, comp = eval_loss_batch(tb, Dataset(X, y), opts)
    orc = Oracle.from_options(opts)
    tol, o_loss, o_comp, _ = loss_tolerance(orc, tb, X, y, rel_bar=1e-10)
    assert np.array_equal(comp, o_comp)
    assert_losses_within(loss, o_loss, comp, tol, "wide f64")


def test_dead_tree_hints_survive_in_place_regrowth():
    """VERDICT r3 #9 (the bug fixed in 58818aa): the dead-tree hint array is epoch-tagged and never
    cleared between calls, so a grown array whose new words happen to equal the next call's epoch marks
    live trees dead.  The debug hook grows it IN PLACE (same address) with exactly those stale words —
    the bug's conditions — and every call must still equal the oracle; with the reallocation detected by
    address instead of capacity, the grown part would keep its stale epochs and this test fails."""
    opts = Options(**C2_OPTS)
    X, y = _c2_data(1 << 17, seed=23)
    d = Dataset(X, y)
    orc = Oracle.from_options(opts)
    ctx = sr_amd.get_context()
    ctx.set_tuning("debug_hint_regrow", 1)
    try:
        for k, n_trees in enumerate((300, 1200, 3500)):  # each call grows the array
            tb = flatten_trees(gen_random_population(n_trees, opts, 5, max_size=30, seed=40 + k), np.float32)
            loss, comp = eval_loss_batch(tb, d, opts)
            o_loss, o_comp = orc.eval_loss_batch(tb, X, y, n_threads=8)
            assert np.array_equal(comp, o_comp), (n_trees, int(np.sum(comp != o_comp)))
            assert 0.2 < comp.mean() < 0.9
            sel = comp & np.isfinite(o_loss)
            assert np.median(_rel(loss[sel], o_loss[sel])) < 1e-6
    finally:
        ctx.set_tuning("debug_hint_regrow", 0)
