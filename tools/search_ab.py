"""Search iterations/s of bench.py's C1 / C3 / C5 configurations (the same data, options and seed), for
A/B runs of the library's latency knobs (set through the SR_AMD_* environment).  One JSON line per
configuration; argv: configurations (default C1 C3 C5), ITERS (env, default 40), and "share" to add
C5's rank-0 share of an 8-rank island-sharded search."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "symbolicregression.jl_amd")]
import numpy as np  # noqa: E402

from sr_amd import Options, equation_search  # noqa: E402


def configs():
    rng = np.random.default_rng(0)
    X1 = rng.standard_normal((2, 100))
    y1 = 2 * np.cos(X1[1]) + X1[0] ** 2 - 2
    o1 = Options(binary_operators=["+", "*", "/", "-"], unary_operators=["cos", "exp"], populations=20)
    rng = np.random.default_rng(11)
    X3 = rng.uniform(0.5, 2.0, (5, 100_000)).astype(np.float32)
    y3 = (X3[0] * X3[1] * X3[2] / (X3[3] * X3[4] ** 2 + 1)).astype(np.float32)
    o3 = Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp", "log"], populations=31)
    o5 = Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp", "log"], populations=32,
                 should_optimize_constants=True)
    return {"C1": (X1, y1, o1), "C3": (X3, y3, o3), "C5": (X3.astype(np.float64), y3.astype(np.float64), o5)}


if __name__ == "__main__":
    args = sys.argv[1:]
    share = "share" in args
    which = [a for a in args if a != "share"] or ["C1", "C3", "C5"]
    iters = int(os.environ.get("ITERS", "40"))
    cf = configs()
    env = {k: v for k, v in os.environ.items() if k.startswith("SR_AMD_")}
    for name in which:
        X, y, o = cf[name]
        runs = [("full", None)] + ([("rank0_of_8", (0, 8))] if share and name == "C5" else [])
        for tag, rs in runs:
            t0 = time.perf_counter()
            res = equation_search(X, y, niterations=iters, options=o, seed=0, _rank_share=rs)
            wall = time.perf_counter() - t0
            print(json.dumps({"config": name, "run": tag, "env": env, "iterations": iters,
                              "iterations_per_s": iters / res.wall_s, "loop_wall_s": res.wall_s, "call_wall_s": wall,
                              "device_calls": res.device_calls, "device_s": res.device_s, "host_s": res.host_s,
                              "us_per_call": res.device_s / max(res.device_calls, 1) * 1e6}), flush=True)
