"""GPU: the elementwise-loss catalog (src/Options.jl:301-328, LossFunctions.jl restated in
csrc/sr_ops.h and in the oracle) — every loss against the oracle on random populations (flags
bit-exact, losses on well-conditioned trees), weighted and SubDataset paths, f64, and the
forward-mode gradient of the smooth ones against the oracle's finite differences.  Only L2/L1 are
pinned by reference tests (test/unit/misc/test_losses.jl:15-33, tests/test_oracle_golden.py); the
others follow the published LossFunctions definitions (parity unpinned beyond the oracle's own
hand-computed points, test_oracle_golden.py::test_loss_catalog_known_answers).
"""
import numpy as np
import pytest

from oracle import Oracle
from parity_util import assert_losses_within, loss_tolerance
from sr_amd import Dataset, Options, SubDataset, eval_grad_batch, eval_loss_batch, flatten_trees, gen_random_population

pytestmark = pytest.mark.gpu

CATALOG = ["L2DistLoss()", "L1DistLoss()", "LPDistLoss{3}()", "LogitDistLoss()", "HuberLoss()", "HuberLoss(0.3)",
           "L1EpsilonInsLoss(0.2)", "L2EpsilonInsLoss(0.2)", "PeriodicLoss(4.0)", "QuantileLoss(0.3)",
           "ZeroOneLoss()", "PerceptronLoss()", "L1HingeLoss()", "L2HingeLoss()", "SmoothedL1HingeLoss(0.5)",
           "ModifiedHuberLoss()", "L2MarginLoss()", "ExpLoss()", "SigmoidLoss()", "DWDMarginLoss(2)"]
OPS = dict(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp", "log"])


def _data(n, seed, dtype, margin=False):
    rng = np.random.default_rng(seed)
    X = rng.standard_normal((4, n)).astype(dtype)
    y = 2 * np.cos(X[3]) + X[0] ** 2 - 2 + 0.1 * rng.standard_normal(n)
    if margin:  # classification targets for the margin-based losses
        y = np.sign(y) + (y == 0)
    return X, y.astype(dtype)


def _rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    with np.errstate(invalid="ignore"):
        return np.where(a == b, 0.0, np.abs(a - b) / np.maximum(np.abs(b), 1e-30))


@pytest.mark.parametrize("spec", CATALOG)
def test_loss_catalog_vs_oracle(spec):
    opts = Options(elementwise_loss=spec, **OPS)
    margin = opts.loss_kind >= 9
    X, y = _data(3000, 1, np.float32, margin)
    tb = flatten_trees(gen_random_population(500, opts, 4, max_size=20, seed=2), np.float32)
    loss, comp = eval_loss_batch(tb, Dataset(X, y), opts)
    orc = Oracle.from_options(opts)
    tol, ol, oc, n_wide = loss_tolerance(orc, tb, X, y, loss_kind=opts.loss_kind, loss_param=opts.loss_param)
    assert np.array_equal(comp, oc), np.nonzero(comp != oc)[0][:10]
    assert np.all(np.isinf(loss[~comp]))
    assert n_wide < 0.3 * comp.sum()
    assert_losses_within(loss, ol, comp, tol, spec)


@pytest.mark.parametrize("spec", ["HuberLoss(0.5)", "QuantileLoss(0.7)", "L2HingeLoss()", "LogitDistLoss()"])
def test_loss_catalog_weighted_gather_f64(spec):
    opts = Options(elementwise_loss=spec, **OPS)
    X, y = _data(2000, 3, np.float64, opts.loss_kind >= 9)
    w = np.random.default_rng(4).uniform(0.5, 2.0, 2000)
    idx = np.random.default_rng(5).integers(0, 2000, 700)
    tb = flatten_trees(gen_random_population(300, opts, 4, max_size=20, dtype=np.float64, seed=6), np.float64)
    loss, comp = eval_loss_batch(tb, SubDataset(Dataset(X, y, weights=w), idx), opts)
    orc = Oracle.from_options(opts)
    # the Float64 bar per tree, every complete tree: 1e-10 relative or 4x its libm spread
    tol, ol, oc, _ = loss_tolerance(orc, tb, X[:, idx], y[idx], w=w[idx], loss_kind=opts.loss_kind,
                                    loss_param=opts.loss_param, rel_bar=1e-10)
    assert np.array_equal(comp, oc)
    assert_losses_within(loss, ol, comp, tol, spec)
    r = _rel(loss[comp], ol[comp])
    assert np.median(r) < 1e-13, spec


@pytest.mark.parametrize("spec", ["HuberLoss(0.5)", "LogitDistLoss()", "LPDistLoss{3}()", "PeriodicLoss(4.0)",
                                  "L2MarginLoss()", "ExpLoss()", "SigmoidLoss()"])
def test_loss_catalog_gradient_vs_finite_differences(spec):
    opts = Options(elementwise_loss=spec, binary_operators=["+", "-", "*"], unary_operators=["cos"])
    X, y = _data(1500, 7, np.float64, opts.loss_kind >= 9)
    tb = flatten_trees(gen_random_population(200, opts, 4, max_size=15, dtype=np.float64, seed=8), np.float64)
    loss, g, comp = eval_grad_batch(tb, Dataset(X, y), opts)
    g_fd, _, comp_o, fd_err = Oracle.from_options(opts).loss_grad_fd(tb, X, y, loss_kind=opts.loss_kind,
                                                                       loss_param=opts.loss_param, with_error=True)
    assert np.array_equal(comp, comp_o)
    co = tb.constant_offsets()
    checked = 0
    for t in np.nonzero(comp)[0]:
        a, b, e = g[co[t]:co[t + 1]], g_fd[co[t]:co[t + 1]], fd_err[co[t]:co[t + 1]]
        if len(a) == 0:
            continue
        scale = max(1.0, float(np.abs(b).max()))
        if e.max() > 1e-6 * scale:
            continue
        assert np.all(np.abs(a - b) <= 1e-6 * scale), (spec, t, a, b)
        checked += 1
    assert checked > 20
