"""Per-tree vs per-instruction interpreter cost (GPU box): 10k copies of chain trees of k binary
instructions (x1 op x2 op x3 ..., every tree complete) over 1M rows; the kernel time against k gives
the fixed cost of a tree on a tile (intercept) and the cost of one dispatched instruction (slope).
Also: a cos / exp / log node per instruction, to price the bodies."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "symbolicregression.jl_amd")]
import numpy as np  # noqa: E402

import sr_amd  # noqa: E402
from sr_amd import Dataset, Options, eval_loss_batch, flatten_trees, parse_expression  # noqa: E402

n = 1 << 20
rng = np.random.default_rng(2)
X = (rng.standard_normal((5, n)) * 0.5 + 1.5).astype(np.float32)  # positive: log stays finite
y = (X[0] * X[1]).astype(np.float32)
ds = Dataset(X, y)
ctx = sr_amd.get_context()
opts = Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp", "log"])


def chain(k, unary=None):
    e = "x1"
    for i in range(k):
        e = f"({e} {'+*-'[i % 3]} x{(i % 4) + 2})"
        if unary:
            e = f"{unary}({e})"
    return e


def run(expr, reps=10000):
    tb = flatten_trees([parse_expression(expr, opts)] * reps, np.float32)
    eval_loss_batch(tb, ds, opts)
    ks = []
    for _ in range(5):
        _, c = eval_loss_batch(tb, ds, opts)
        ks.append(ctx.last_kernel_ms()[0])
    return float(np.median(ks)), bool(c.all())


for label, u in (("arith", None), ("cos", "cos"), ("exp", "exp"), ("log", "log"), ("div", "div"), ("logexp", "logexp")):
    for k in (1, 2, 4, 8, 16):
        if u in ("exp", "logexp") and k > 4:
            continue
        e = chain(k, u if u in ("cos", "log") else None)
        if u == "exp":  # exp of a bounded argument: cos inside keeps it finite
            e = "x1"
            for i in range(k):
                e = f"exp(cos({e} * x{(i % 4) + 2}))"
        if u == "logexp":  # log of a positive argument: the exp chain above with a log on each level
            e = "x1"
            for i in range(k):
                e = f"log(exp(cos({e} * x{(i % 4) + 2})))"
        if u == "div":  # x1 / x2 / x3 ...: the Julia-faithful Float32 division (X > 0 almost surely)
            e = "x1"
            for i in range(k):
                e = f"({e} / x{(i % 4) + 2})"
        ms, comp = run(e)
        print(f"{label:6s} k={k:2d} kernel={ms:8.3f}ms  per-tree-row={ms / 10000 / n * 1e12:7.2f}ps complete={comp}  {e[:60]}",
              flush=True)
