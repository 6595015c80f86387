"""Round 6 debugging: one tree's loss under the fold vs numpy's sequential fold (analysis only)."""
import os
import sys

import numpy as np

sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "symbolicregression.jl_amd")]
import sr_amd  # noqa: E402
from sr_amd import Dataset, Options, eval_loss_batch, flatten_trees, parse_expression  # noqa: E402

opts = Options(binary_operators=["+", "*", "-", "/"], unary_operators=["cos", "exp", "sin"])
ctx = sr_amd.get_context()
for dtype in (np.float64, np.float32):
    for n in (300, 3001, 100_000):
        rng = np.random.default_rng(0)
        X = rng.standard_normal((3, n)).astype(dtype)
        y = (X[0] * 2 + 0.1 * rng.standard_normal(n)).astype(dtype)
        tb = flatten_trees([parse_expression("3.2 * x1", opts), parse_expression("x1 * x2", opts)], dtype)
        pred = [dtype(dtype(3.2) * X[0]), X[0] * X[1]]
        for rf in (1, 0):
            ctx.set_tuning("ref_fold", rf)
            loss, comp = eval_loss_batch(tb, Dataset(X, y), opts)
            refs = []
            for p in pred:
                l = ((p - y) ** 2).astype(dtype)
                f = l[0]
                for v in l[1:]:
                    f = dtype(f + v)
                refs.append(dtype(f / dtype(n)))
            print(dtype.__name__, n, "ref_fold", rf, "loss", loss, "ref", refs, "fold", ctx.last_ref_fold(), flush=True)
ctx.set_tuning("ref_fold", 1)
