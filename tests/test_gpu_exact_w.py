"""GPU: the exact-sum pass (Julia-order isfinite(sum) of the checked arrays of BIG trees) at four
waves per workgroup (`exact_w` 4, the default) against one wave (`exact_w` 1, the previous layout).

The four waves of a workgroup share one staged row range and fold their own listed trees, so the
flags must be the same bits under both layouts and equal to the oracle's. `exact_g` forces several
listed trees per workgroup, which small row counts would otherwise not reach. The adversarial
columns of tests/test_jsum.py put the verdicts where an f64 sum and Julia's Float32 pairwise sum
disagree."""
import numpy as np
import pytest

import sr_amd
from oracle import Oracle
from sr_amd import Dataset, Options, eval_loss_batch, flatten_trees, parse_expression

pytestmark = pytest.mark.gpu

EXPRS = ["x1 * 1.0", "(x1 * 1.0) + (x2 * 0.0)", "cos(x2) * (x1 * x3)", "(x1 - x2) / (x3 * 1.0)", "x1 + x2",
         "(x1 * 0.5) + (x1 * 0.5)", "x1 * x3", "(x3 * x1) - x2", "x1 * 2.0", "(x1 + x2) * 1.0"]


def _columns():
    from test_jsum import cases

    return {k: v for k, v in cases().items() if k not in ("one", "fifteen")}


def _run(tb, ds, opts, w, g):
    ctx = sr_amd.get_context()
    ctx.set_tuning("exact_w", w)
    ctx.set_tuning("exact_g", g)
    try:
        return eval_loss_batch(tb, ds, opts)
    finally:
        ctx.set_tuning("exact_w", 4)
        ctx.set_tuning("exact_g", 0)


@pytest.mark.parametrize("name", list(_columns()))
def test_exact_pass_four_waves_equals_one_and_oracle(name):
    col = _columns()[name]
    n = len(col)
    X = np.stack([col, np.zeros(n, np.float32), np.ones(n, np.float32)]).astype(np.float32)
    y = np.zeros(n, dtype=np.float32)
    opts = Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos"])
    tb = flatten_trees([parse_expression(e, opts) for e in EXPRS], np.float32)
    ds = Dataset(X, y)
    _, oc = Oracle.from_options(opts).eval_loss_batch(tb, X, y, n_threads=4)
    results = {}
    for w, g in ((1, 0), (4, 0), (4, 4), (4, 8), (1, 8)):
        loss, comp = _run(tb, ds, opts, w, g)
        assert list(comp) == list(oc), (name, w, g, list(zip(EXPRS, comp, oc)))
        results[(w, g)] = loss
    ref = results[(1, 0)]
    for key, loss in results.items():  # (the losses come from the main pass: the same bits)
        assert np.array_equal(loss.view(np.uint32), ref.view(np.uint32)), (name, key)
