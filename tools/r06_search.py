"""Round 6: the C3 search's rate under the current environment (one line; analysis only).
usage: python tools/r06_search.py [iters] [c3|c1|c5]"""
import os
import sys
import time

import numpy as np

sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "symbolicregression.jl_amd")]
from sr_amd import Options, equation_search  # noqa: E402

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 20
which = sys.argv[2] if len(sys.argv) > 2 else "c3"
rng = np.random.default_rng(11)
X3 = rng.uniform(0.5, 2.0, (5, 100_000)).astype(np.float32)
y3 = (X3[0] * X3[1] * X3[2] / (X3[3] * X3[4] ** 2 + 1)).astype(np.float32)
if which == "c3":
    X, y = X3, y3
    o = Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp", "log"], populations=31)
elif which == "c5":
    X, y = X3.astype(np.float64), y3.astype(np.float64)
    o = Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp", "log"], populations=32,
                should_optimize_constants=True)
else:
    rng = np.random.default_rng(0)
    X = rng.standard_normal((2, 100))
    y = 2 * np.cos(X[1]) + X[0] ** 2 - 2
    o = Options(binary_operators=["+", "*", "/", "-"], unary_operators=["cos", "exp"], populations=20)
equation_search(X, y, niterations=2, options=o, seed=0)  # warm
t0 = time.perf_counter()
res = equation_search(X, y, niterations=iters, options=o, seed=0)
wall = time.perf_counter() - t0
print(f"{which} env={os.environ.get('R06_TAG', '')} it/s {iters / wall:.2f} calls {res.device_calls} "
      f"device_s {res.device_s:.3f} per_call_us {res.device_s / max(res.device_calls, 1) * 1e6:.1f} "
      f"host_s {res.host_s:.3f} best {min(m.loss for m in res.pareto_frontier):.4g}", flush=True)
