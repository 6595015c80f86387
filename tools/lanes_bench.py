"""GPU: search throughput (C1, C3 as bench.py builds them) vs the number of scoring lanes (device
contexts + host threads the islands are split over).  usage: python tools/lanes_bench.py [iters] [lanes...]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if os.environ.get("LANES_KERNEL_TIMES") == "1":
    os.environ["SR_AMD_SEARCH_KERNEL_TIMES"] = "1"
sys.path[:0] = [os.path.join(ROOT, "symbolicregression.jl_amd")]
import numpy as np  # noqa: E402

from sr_amd import Options, equation_search  # noqa: E402


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    lanes = [int(v) for v in sys.argv[2:]] or [1, 2, 3, 4]
    rng = np.random.default_rng(0)
    X1 = rng.standard_normal((2, 100))
    y1 = 2 * np.cos(X1[1]) + X1[0] ** 2 - 2
    o1 = Options(binary_operators=["+", "*", "/", "-"], unary_operators=["cos", "exp"], populations=20)
    rng = np.random.default_rng(11)
    X3 = rng.uniform(0.5, 2.0, (5, 100_000)).astype(np.float32)
    y3 = (X3[0] * X3[1] * X3[2] / (X3[3] * X3[4] ** 2 + 1)).astype(np.float32)
    o3 = Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp", "log"], populations=31)
    for name, X, y, o in (("c1", X1, y1, o1), ("c3", X3, y3, o3)):
        equation_search(X, y, niterations=1, options=o, seed=0)  # warm-up
        for L in lanes:
            t0 = time.perf_counter()
            res = equation_search(X, y, niterations=iters, options=o, seed=0, scoring_lanes=L)
            wall = time.perf_counter() - t0
            print(json.dumps({"config": name, "lanes": L, "iterations": iters, "it_per_s": iters / wall,
                              "calls": res.device_calls, "device_wall_per_call_us": res.device_s / res.device_calls * 1e6,
                              "kernel_busy_per_call_us": res.kernel_s / res.device_calls * 1e6,
                              "host_s": res.host_s, "wall_s": wall}), flush=True)


if __name__ == "__main__":
    main()
