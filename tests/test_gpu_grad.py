"""GPU: batched forward-mode loss gradient with respect to tree constants (sr_eval_grad_batch).

Mirrors the reference's constant-derivative tests (test/integration/ad/zygote/test_derivatives.jl:
91-123: d(3.2*x1)/dc = x1 and the two-constant "equation5" expression, constant order :127-155)
re-expressed as gradients of the L2 loss with closed forms, plus random populations against
central finite differences of the f64 CPU oracle (the gradient-free objective Optim's BFGS
differentiates by default, src/ConstantOptimization.jl:77-116).
"""
import numpy as np
import pytest

from oracle import Oracle
from sr_amd import Dataset, Options, eval_grad_batch, flatten_trees, gen_random_population, parse_expression

pytestmark = pytest.mark.gpu


def _data(n, seed, dtype):
    rng = np.random.default_rng(seed)
    X = rng.standard_normal((3, n)).astype(dtype)
    y = (2 * np.cos(X[2]) + X[0] ** 2 - 2 + 0.1 * rng.standard_normal(n)).astype(dtype)
    return X, y


@pytest.mark.parametrize("dtype,tol", [(np.float64, 1e-12), (np.float32, 2e-5)])
def test_known_answer_linear(dtype, tol):
    opts = Options(binary_operators=["+", "*", "-", "/"], unary_operators=["cos", "exp", "sin"])
    X, y = _data(3001, 0, dtype)
    tb = flatten_trees([parse_expression("3.2 * x1", opts)], dtype)
    loss, g, comp = eval_grad_batch(tb, Dataset(X, y), opts)
    x1, yy = X[0].astype(np.float64), y.astype(np.float64)
    ref = np.mean(2 * (3.2 * x1 - yy) * x1)  # d/dc mean((c*x1 - y)^2) at c = 3.2
    assert comp[0] and g.shape == (1,)
    assert abs(g[0] - ref) <= tol * max(1.0, abs(ref))
    assert abs(loss[0] - np.mean((np.float64(dtype(3.2)) * x1 - yy) ** 2)) <= 1e-5 * loss[0]


@pytest.mark.parametrize("dtype,tol", [(np.float64, 1e-10), (np.float32, 1e-4)])
def test_known_answer_equation5(dtype, tol):
    # equation5 (test_derivatives.jl:101-123) with the catalog's ops: pow_abs2(x1,x2) = abs(x1)^x2,
    # custom_cos(x) = cos(x)^2 -> square(cos(x))
    opts = Options(binary_operators=["+", "*", "-", "/", "^"], unary_operators=["cos", "abs", "square"])
    X, y = _data(2000, 1, dtype)
    X[0] = np.where(np.abs(X[0]) < 0.1, 0.5, X[0])  # keep c2 / x1 tame
    c1, c2 = 2.1, -3.2
    tree = parse_expression("((abs(x1) ^ x2) + x3) + (square(cos(2.1 + x3)) + (-3.2 / x1))", opts)
    tb = flatten_trees([tree], dtype)
    loss, g, comp = eval_grad_batch(tb, Dataset(X, y), opts)
    x1, x2, x3, yy = (v.astype(np.float64) for v in (X[0], X[1], X[2], y))
    pred = np.abs(x1) ** x2 + x3 + np.cos(c1 + x3) ** 2 + c2 / x1
    d = 2 * (pred - yy)
    ref = np.array([np.mean(d * (-2 * np.cos(c1 + x3) * np.sin(c1 + x3))), np.mean(d / x1)])
    assert comp[0]
    np.testing.assert_allclose(g, ref, rtol=tol, atol=tol * np.abs(ref).max())


def test_population_f64_vs_finite_differences():
    opts = Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp", "log", "sin"])
    X, y = _data(1500, 2, np.float64)
    trees = gen_random_population(400, opts, 3, seed=5)
    tb = flatten_trees(trees, np.float64)
    loss, g, comp = eval_grad_batch(tb, Dataset(X, y), opts)
    g_fd, loss_o, comp_o, fd_err = Oracle.from_options(opts).loss_grad_fd(tb, X, y, with_error=True)
    assert np.array_equal(comp, comp_o)
    co = tb.constant_offsets()
    n_checked = 0
    for t in np.nonzero(comp)[0]:
        a, b, e = g[co[t]:co[t + 1]], g_fd[co[t]:co[t + 1]], fd_err[co[t]:co[t + 1]]
        if len(a) == 0:
            continue
        scale = max(1.0, float(np.abs(b).max()))
        if e.max() > 1e-6 * scale:  # finite differences themselves unreliable (strong curvature)
            continue
        assert np.all(np.abs(a - b) <= 1e-6 * scale), (t, a, b)
        n_checked += 1
    assert n_checked > 50
    # incomplete trees: L(Inf) and a zero gradient
    for t in np.nonzero(~comp)[0]:
        assert np.isinf(loss[t]) and np.all(g[co[t]:co[t + 1]] == 0)


def test_population_f32_close_to_f64():
    # same f32-representable data and constants in both precisions; trees whose f32 loss already
    # differs from the f64 one (ill-conditioned evaluation) are not a gradient question
    opts = Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp"])
    X32, y32 = _data(4096, 3, np.float32)
    tb32 = flatten_trees(gen_random_population(300, opts, 3, seed=6), np.float32)
    l32, g32, c32 = eval_grad_batch(tb32, Dataset(X32, y32), opts)
    l64, g64, c64 = eval_grad_batch(tb32.astype(np.float64), Dataset(X32.astype(np.float64), y32.astype(np.float64)), opts)
    co = tb32.constant_offsets()
    checked = bad = 0
    for t in np.nonzero(c32 & c64)[0]:  # (f32 / f64 overflow thresholds differ)
        a, b = g32[co[t]:co[t + 1]].astype(np.float64), g64[co[t]:co[t + 1]]
        if len(b) == 0 or not abs(float(l32[t]) - l64[t]) <= 1e-5 * abs(l64[t]):
            continue
        checked += 1
        scale = max(1.0, float(np.abs(b).max()))
        bad += int(not np.all(np.abs(a - b) <= 1e-2 * scale))
    assert checked > 100 and bad <= 0.04 * checked, (checked, bad)


def test_many_constants_weighted_gather_l1():
    # more constants than one tangent pass holds (16), weights, a SubDataset view and L1DistLoss
    opts = Options(binary_operators=["+", "*"], unary_operators=["cos"], elementwise_loss="L1DistLoss")
    X, y = _data(1000, 4, np.float64)
    w = np.random.default_rng(9).uniform(0.5, 2.0, 1000)
    expr = " + ".join(f"{0.1 * (k + 1)} * cos(x{1 + k % 3} + {0.05 * k})" for k in range(10))  # 20 constants
    tb = flatten_trees([parse_expression(expr, opts)], np.float64)
    idx = np.random.default_rng(10).integers(0, 1000, 300)
    ds = Dataset(X, y, weights=w)
    from sr_amd import SubDataset

    loss, g, comp = eval_grad_batch(tb, SubDataset(ds, idx), opts)
    g_fd, _, _ = Oracle.from_options(opts).loss_grad_fd(tb, X[:, idx], y[idx], w[idx], loss_kind=1)
    assert comp[0] and len(g) == 20
    np.testing.assert_allclose(g, g_fd, rtol=1e-5, atol=1e-6)


def test_bfgs_batch_recovers_constants():
    # batched BFGS / Newton (src/ConstantOptimization.jl:29-116) on trees whose optimum is known
    from sr_amd import optimize_constants_batch

    opts = Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp"])
    rng = np.random.default_rng(11)
    X = rng.standard_normal((3, 2000)).astype(np.float64)
    y = 3.0 * X[0] + 1.5
    trees = [parse_expression("1.0 * x1 + 1.0", opts),      # BFGS, 2 constants -> (3, 1.5)
             parse_expression("x1 * 1.0", opts),             # Newton, 1 constant -> 3 (+ residual)
             parse_expression("cos(x2) * 0.5", opts),        # nothing to gain much
             parse_expression("x1 * x2", opts)]              # no constants
    tb = flatten_trees(trees, np.float64)
    ds = Dataset(X, y)
    from sr_amd import eval_loss_batch

    l0, _ = eval_loss_batch(tb, ds, opts)
    new_tb, losses, improved, n_evals = optimize_constants_batch(tb, ds, opts, np.random.default_rng(0))
    c = new_tb.get_constants()
    assert improved[0] and improved[1] and not improved[3]
    np.testing.assert_allclose(c[0:2], [3.0, 1.5], rtol=1e-6)
    assert abs(c[2] - 3.0) < 0.1
    assert losses[0] < 1e-10 and np.all(losses <= l0 + 1e-12)
    assert np.all(n_evals[:2] > 1)
    # a not-improved tree keeps its constants exactly
    for k in np.nonzero(~improved)[0]:
        co = tb.constant_offsets()
        np.testing.assert_array_equal(new_tb.get_constants()[co[k]:co[k + 1]], tb.get_constants()[co[k]:co[k + 1]])


def test_f_calls_limit_is_honoured():
    """Optim.Options' f_calls_limit crosses the C ABI (sr_optimize_constants_batch) and
    the device optimiser honours it: a limit of 3 objective calls stops every start after its first
    iteration (each costs >= 3 calls), exactly as iterations = 1 does — constants, losses and num_evals
    bit for bit — while the default limit (10_000) equals no limit."""
    from sr_amd import optimize_constants_batch

    opts = Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp"])
    rng = np.random.default_rng(12)
    X = rng.standard_normal((3, 4000)).astype(np.float64)
    y = 3.0 * X[0] * np.cos(X[1] * 0.7) + 1.5
    trees = [parse_expression(e, opts) for e in ("1.0 * x1 + 1.0", "x1 * cos(x2 * 0.5) * 2.0 + 1.0", "x1 * 1.0",
                                                 "exp(x3 * 0.1) * 0.3 + x1 * 2.5")]
    tb = flatten_trees(trees, np.float64)
    ds = Dataset(X, y)
    run = lambda **kw: optimize_constants_batch(tb, ds, opts, np.random.default_rng(4), **kw)  # noqa: E731
    lim, one = run(f_calls_limit=3), run(iterations=1)
    for a, b in zip(lim, one):
        a, b = (a.val, b.val) if hasattr(a, "val") else (a, b)
        assert np.array_equal(a, b)
    full, dflt = run(f_calls_limit=0), run()
    assert np.array_equal(full[0].val, dflt[0].val) and np.array_equal(full[3], dflt[3])
    assert np.all(lim[3] <= full[3]) and np.any(lim[3] < full[3])
    assert np.any(full[1] < lim[1])


def test_grad_f64_many_features_deep_trees_weighted():
    """Float64 with 10 features, weights, maxsize 30 and unary operators — trees of
    stack depth 3 and two-constant trees in one batch.  The 8-rows-per-lane buckets' LDS operand stacks
    do not fit 160 KiB there; those buckets must fall back to one row per lane instead of failing, and
    the gradient must still match central finite differences of the f64 oracle."""
    opts = Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp", "sin"])
    rng = np.random.default_rng(12)
    nf = 10
    X = rng.standard_normal((nf, 1500))
    y = np.cos(X[0]) + X[1] * X[2]
    w = rng.uniform(0.5, 2.0, 1500)
    trees = gen_random_population(300, opts, nf, max_size=30, seed=13)
    trees += [parse_expression("cos(cos(x1 * 1.5) + sin(x2 * 0.5)) * (x3 + (x4 - x5 * x6))", opts)]
    tb = flatten_trees(trees, np.float64)
    loss, g, comp = eval_grad_batch(tb, Dataset(X, y, weights=w), opts)
    g_fd, _, comp_o, fd_err = Oracle.from_options(opts).loss_grad_fd(tb, X, y, w, with_error=True)
    assert np.array_equal(comp, comp_o)
    co = tb.constant_offsets()
    checked = 0
    for t in np.nonzero(comp)[0]:
        a, b, e = g[co[t]:co[t + 1]], g_fd[co[t]:co[t + 1]], fd_err[co[t]:co[t + 1]]
        if len(a) == 0:
            continue
        scale = max(1.0, float(np.abs(b).max()))
        if e.max() > 1e-6 * scale or not loss[t] < 1e8:
            # (finite differences of a loss of 1e25 — exp(exp(x)) terms — resolve nothing: both
            # steps see the same loss bits and report a zero gradient with a zero error estimate)
            continue
        # (10 features and weights: the finite differences' own rounding error is ~1e-6 here)
        assert np.all(np.abs(a - b) <= 2e-5 * scale), (t, a, b)
        checked += 1
    assert checked > 50


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_gradients_independent_of_rows_per_lane(dtype):
    """The gradient kernel's rows per lane is a tuning choice (sr_set_tuning "grad_rows"): its row
    blocks cover the same rows whatever the choice and each lane accumulates its rows in order, so the
    gradients are bit-identical for every choice — also with FULL-tier operators (their row callees),
    weights, a non-L2 loss and every tangent bucket.  Likewise the work items' order (sr_set_tuning
    "grad_sort": by program cost, or in tree order)."""
    import sr_amd

    rng = np.random.default_rng(8)
    n = 30_001
    X = rng.uniform(0.5, 2.0, (4, n)).astype(dtype)
    y = (X[0] * X[1] / (X[2] + 1) + np.cos(X[3])).astype(dtype)
    w = (0.5 + rng.random(n)).astype(dtype)
    ctx = sr_amd.get_context()
    for kw, loss in ((dict(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp", "log", "sin"]), None),
                     (dict(binary_operators=["+", "*", "/", "^", "max"], unary_operators=["tanh", "sqrt", "atan"]),
                      "L1DistLoss")):
        opts = Options(**kw, **({"elementwise_loss": loss} if loss else {}))
        trees = gen_random_population(400, opts, 4, max_size=25, dtype=dtype, seed=8)
        tb = flatten_trees(trees, dtype)
        ds = Dataset(X, y, weights=w)
        ref = None
        try:
            for rows in (0, 1, 2, 4, 8):
                ctx.set_tuning("grad_rows", rows)
                l, g, c = eval_grad_batch(tb, ds, opts)
                if ref is None:
                    ref = (l, g, c)
                    assert c.mean() > 0.2
                    continue
                assert np.array_equal(c, ref[2]), rows
                assert np.array_equal(g.view(np.uint8), ref[1].view(np.uint8)), (rows, kw)
            ctx.set_tuning("grad_rows", 0)
            ctx.set_tuning("grad_sort", 0)
            l, g, c = eval_grad_batch(tb, ds, opts)
            assert np.array_equal(c, ref[2])
            assert np.array_equal(g.view(np.uint8), ref[1].view(np.uint8)), ("unsorted", kw)
        finally:
            ctx.set_tuning("grad_rows", 0)
            ctx.set_tuning("grad_sort", 1)
