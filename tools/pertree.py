"""Per-tree overhead probe: populations of identical tiny trees (kernel ms per tree-tile)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "symbolicregression.jl_amd")]
import numpy as np
import sr_amd
from sr_amd import Options, Dataset, flatten_trees, parse_expression, eval_loss_batch

n = 1 << 20
rng = np.random.default_rng(2)
X = rng.standard_normal((5, n)).astype(np.float32)
y = (2 * np.cos(X[3]) + X[0] ** 2 - 2).astype(np.float32)
ds = Dataset(X, y)
ctx = sr_amd.get_context()
opts = Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp", "log"])
for expr in ["x1", "x1 * 2.0", "x1 * x2 + x3", "(x1 * x2 + x3) * (x4 - x5 * 3.0)",
             "((x1 * x2 + x3) * (x4 - x5 * 3.0) + x1 * 1.5) * (x2 - 0.5) + x3 * x4 * x5"]:
    t = parse_expression(expr, opts)
    for nt in (2000, 10000):
        b = flatten_trees([t] * nt, np.float32)
        eval_loss_batch(b, ds, opts)
        ks = []
        for _ in range(5):
            eval_loss_batch(b, ds, opts)
            ks.append(ctx.last_kernel_ms()[0])
        k = float(np.median(ks))
        tile_evals = nt * (n // 512)
        # wave-cycles per tree-tile: kernel time x (256 CUs x 20 resident waves) x 2.4 GHz / tree-tiles
        print(f"{expr[:40]:40s} nodes={t.count_nodes():3d} trees={nt:6d} kernel={k:7.3f} ms "
              f"wave-cycles/tree-tile={k * 1e-3 * 256 * 20 * 2.4e9 / tile_evals:8.0f}", flush=True)
