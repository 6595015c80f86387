"""CPU: host-side native pieces that need no device — the library's random-population generator
(`sr_gen_random_population`, C4's 100k trees) and the batched constant optimiser driven by CPU
scorers (`sr_optimize_constants_callbacks`: the same BFGS / Newton code the device path runs,
src/ConstantOptimization.jl:29-116), scored by the oracle."""
import numpy as np
import pytest

from oracle import Oracle, loss_grad_forward
from sr_amd import Options, flatten_trees, gen_random_batch, gen_random_population, parse_expression, string_tree
from sr_amd.constant_optimization import optimize_constants_callbacks

OPS = dict(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp", "log"])


def test_native_population_matches_generator_distribution():
    """gen_random_tree_fixed_size (src/MutationFunctions.jl:441-471) with node_count ~ U{1..30}: the
    native generator's population has the Python generator's statistics (mean size, unary : binary
    ratio = nuna : nbin = 3 : 4, leaves half constants), is seeded, and every tree parses back."""
    opts = Options(**OPS)
    a = gen_random_batch(20_000, opts, 5, seed=4)
    b = gen_random_batch(20_000, opts, 5, seed=4)
    assert np.array_equal(a.offsets, b.offsets) and np.array_equal(a.val, b.val)
    ref = flatten_trees(gen_random_population(5_000, opts, 5, seed=9), np.float32)
    for tb in (a, ref):
        sizes = np.diff(tb.offsets)
        assert 14.5 < sizes.mean() < 16.5
        assert sizes.min() >= 1 and sizes.max() <= 30
        un, bi = np.sum(tb.degree == 1), np.sum(tb.degree == 2)
        assert 0.6 < un / bi < 0.9
        leaves = tb.degree == 0
        assert 0.45 < tb.constant[leaves].mean() < 0.55
        assert np.all((tb.feature[leaves & (tb.constant == 0)] >= 1) & (tb.feature[leaves & (tb.constant == 0)] <= 5))
    for k in range(50):
        assert string_tree(a.tree(k), opts.operators)


def _scorers(opts, X, y):
    orc = Oracle.from_options(opts)

    def lossf(b, rows):
        l, c = orc.eval_loss_batch(b, X, y, accum="f64", n_threads=4)
        return np.where(c, l, np.inf)

    def gradf(b, rows):
        g, l, c = loss_grad_forward(orc, b, X, y)
        return np.where(c, l, np.inf), g
    return lossf, gradf


def test_callback_optimiser_reaches_known_optima():
    """BFGS (several constants) and Newton (one constant) from perturbed starts approach the exact
    optimum; the start loss is never made worse; the restarts are seeded (same seed, same result)."""
    rng = np.random.default_rng(3)
    X = rng.uniform(0.5, 2.0, (3, 500))
    opts = Options(**OPS)
    cases = [(2.5 * X[0] * X[1] / (X[2] + 0.75), "1.9 * x1 * x2 / (x3 + 0.5)", [2.5, 0.75], 1e-5),     # BFGS
             (2.5 * X[0] * X[1] / (X[2] + 0.75), "x1 * x2 / (x3 * 0.5 + 0.2)", [0.4, 0.3], 1e-12),    # BFGS
             (2.5 * X[0] * X[1] / X[2], "1.3 * x1 * x2 / x3", [2.5], 1e-12)]                           # Newton
    for y, expr, want, bar in cases:
        lossf, gradf = _scorers(opts, X, y)
        tb = flatten_trees([parse_expression(expr, opts), parse_expression("cos(x1) + 0.3", opts)], np.float64)
        start = lossf(tb, None)
        out, loss, improved, f_calls = optimize_constants_callbacks(tb, lossf, gradf, seed=11)
        assert np.all(loss <= start) and improved[0] and f_calls[0] > 0, expr
        # 8 iterations (the reference's default optimizer_iterations)
        assert loss[0] < bar * start[0], (expr, loss[0], start[0])
        c0 = out.val[out.offsets[0]:out.offsets[1]][out.constant_mask()[out.offsets[0]:out.offsets[1]]]
        np.testing.assert_allclose(c0, want, rtol=1e-3)
        again = optimize_constants_callbacks(tb, lossf, gradf, seed=11)
        assert np.array_equal(again[1], loss) and np.array_equal(again[0].val, out.val)


def test_callback_optimiser_items_independent_of_batch():
    """The batched optimiser runs every (tree, start) item on its own values: without
    restarts (no random draws), each tree's constants, loss and f_calls are the same optimised alone
    or in one batch with BFGS and Newton members of other shapes."""
    rng = np.random.default_rng(5)
    X = rng.uniform(0.5, 2.0, (3, 400))
    y = 2.5 * X[0] * X[1] / (X[2] + 0.75)
    opts = Options(**OPS)
    lossf, gradf = _scorers(opts, X, y)
    exprs = ["1.9 * x1 * x2 / (x3 + 0.5)", "1.3 * x1 * x2 / x3", "cos(x1 * 0.7) + x2 * 1.1",
             "x1 * x2 / (x3 * 0.5 + 0.2)", "exp(x3 * -0.3) * 2.0"]
    trees = [parse_expression(e, opts) for e in exprs]
    tb = flatten_trees(trees, np.float64)
    out, loss, improved, f_calls = optimize_constants_callbacks(tb, lossf, gradf, nrestarts=0)
    for k, t in enumerate(trees):
        one = flatten_trees([t], np.float64)
        o1, l1, i1, f1 = optimize_constants_callbacks(one, lossf, gradf, nrestarts=0)
        assert l1[0] == loss[k] and i1[0] == improved[k] and f1[0] == f_calls[k], exprs[k]
        assert np.array_equal(o1.val, out.val[out.offsets[k]:out.offsets[k + 1]]), exprs[k]


def test_callback_optimiser_honours_f_calls_limit():
    """Optim.Options' f_calls_limit (src/Options.jl:988-997, passed through the C ABI): a start stops
    after the iteration at whose end its objective calls reach the limit.  Every iteration costs at
    least three calls (value + gradient, one line-search trial, value + gradient at the new point), so
    a limit of 3 stops every start after its first iteration — exactly what iterations = 1 gives; the
    default limit (10_000) never binds at 8 iterations."""
    rng = np.random.default_rng(8)
    X = rng.uniform(0.5, 2.0, (3, 300))
    y = 2.5 * X[0] * X[1] / (X[2] + 0.75)
    opts = Options(**OPS)
    lossf, gradf = _scorers(opts, X, y)
    exprs = ["1.9 * x1 * x2 / (x3 + 0.5)", "1.3 * x1 * x2 / x3", "cos(x1 * 0.7) + x2 * 1.1",
             "x1 * x2 / (x3 * 0.5 + 0.2)"]
    tb = flatten_trees([parse_expression(e, opts) for e in exprs], np.float64)
    lim = optimize_constants_callbacks(tb, lossf, gradf, seed=5, f_calls_limit=3)
    one = optimize_constants_callbacks(tb, lossf, gradf, seed=5, iterations=1)
    full = optimize_constants_callbacks(tb, lossf, gradf, seed=5)
    dflt = optimize_constants_callbacks(tb, lossf, gradf, seed=5, f_calls_limit=10_000)
    assert np.array_equal(lim[0].val, one[0].val) and np.array_equal(lim[1], one[1]) and np.array_equal(lim[3], one[3])
    assert np.array_equal(dflt[0].val, full[0].val) and np.array_equal(dflt[3], full[3])
    assert np.all(lim[3] <= full[3]) and np.sum(lim[3] < full[3]) >= 3  # (Newton's tree converges in one)
    assert np.any(full[1] < lim[1])


def test_non_bfgs_optimizer_is_not_run_on_the_device():
    """A non-default optimizer_algorithm (the reference accepts NelderMead, src/Options.jl:738-746) is
    never replaced by the device's BFGS: the Python mirror refuses it (the Julia glue's
    device_optimizer gate hands it to the reference's optimize_constants)."""
    from sr_amd.constant_optimization import device_optimizer_supported, optimize_constants_batch

    assert device_optimizer_supported(Options(**OPS))
    nm = Options(**OPS, optimizer_algorithm="NelderMead")
    assert not device_optimizer_supported(nm)
    with pytest.raises(NotImplementedError):
        optimize_constants_batch([parse_expression("x1 * 2.0", nm)], None, nm)
    with pytest.raises(ValueError):
        Options(**OPS, optimizer_algorithm="LBFGS")
