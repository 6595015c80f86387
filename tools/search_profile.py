"""Per-lane timings of a search (SR_AMD_SEARCH_PROFILE=1: the engine prints, per lane and iteration,
the regularised-evolution cycles and the constant optimisation with their scoring calls).

usage: python tools/search_profile.py [C3|C5] [lanes ...]   (default C3, 4 lanes)"""
import os, sys, time
os.environ["SR_AMD_SEARCH_PROFILE"] = "1"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "symbolicregression.jl_amd")]
import numpy as np  # noqa: E402
from sr_amd import Options, equation_search  # noqa: E402

args = sys.argv[1:]
cfg = args.pop(0) if args and args[0] in ("C3", "C5") else "C3"
rng = np.random.default_rng(11)
X = rng.uniform(0.5, 2.0, (5, 100_000)).astype(np.float32)
y = (X[0] * X[1] * X[2] / (X[3] * X[4] ** 2 + 1)).astype(np.float32)
if cfg == "C5":  # bench.py's C5: Float64, 32 populations, constant optimisation
    X, y = X.astype(np.float64), y.astype(np.float64)
    o = Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp", "log"], populations=32,
                should_optimize_constants=True)
else:
    o = Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp", "log"], populations=31)
for lanes in [int(v) for v in args] or [4]:
    t0 = time.perf_counter()
    res = equation_search(X, y, niterations=3, options=o, seed=0, scoring_lanes=lanes)
    print(f"{cfg} lanes={lanes} wall {time.perf_counter() - t0:.3f} s for 3 iterations, calls {res.device_calls}, "
          f"device {res.device_s:.3f} s host {res.host_s:.3f} s (summed over lanes)", file=sys.stderr, flush=True)
