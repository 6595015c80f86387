"""Search throughput (BASELINE.json metric part 2, "search iterations/sec"): C1 README example and a
bounded C3 run.  Iterations/sec counts completed s_r_cycles (one per island per iteration,
src/SymbolicRegression.jl:1091) per wall second.  Prints one JSON line per config."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "symbolicregression.jl_amd")]
import numpy as np  # noqa: E402

from sr_amd import Options, equation_search  # noqa: E402


def run(name, X, y, opts, niterations):
    t0 = time.perf_counter()
    res = equation_search(X, y, niterations=niterations, options=opts, seed=0,
                          scoring_lanes=int(os.environ.get("SR_SEARCH_LANES", "4")))
    wall = time.perf_counter() - t0
    best = min(res.pareto_frontier, key=lambda m: m.loss)
    print(json.dumps({"config": name, "islands": opts.populations, "iterations": niterations,
                      "s_r_cycles": res.s_r_cycles, "wall_s": wall,
                      "s_r_cycles_per_s": res.s_r_cycles / wall, "iterations_per_s": niterations / wall,
                      "device_calls": res.device_calls, "device_s": res.device_s, "host_s": res.host_s,
                      "device_fraction": res.device_s / wall, "num_evals": res.num_evals, "best_loss": float(best.loss)}),
          flush=True)


if __name__ == "__main__":
    which = sys.argv[1:] or ["C1", "C3"]
    if "C1" in which:
        rng = np.random.default_rng(0)
        X = rng.standard_normal((2, 100))
        y = 2 * np.cos(X[1]) + X[0] ** 2 - 2
        opts = Options(binary_operators=["+", "*", "/", "-"], unary_operators=["cos", "exp"], populations=20)
        run("C1 README example (X=randn(2,100) f64, 20 populations, default options)", X, y, opts,
            int(os.environ.get("C1_ITERS", "40")))
    if "C3" in which:
        rng = np.random.default_rng(1)
        X = rng.uniform(1, 5, size=(5, 100_000)).astype(np.float32)
        y = (X[0] * X[1] * X[2] / (X[3] * X[4] ** 2 + 1)).astype(np.float32)
        opts = Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp"])
        run("C3 Feynman-style 5 features x 100k rows f32 (31 populations, default options)", X, y, opts,
            int(os.environ.get("C3_ITERS", "5")))
    if "C5" in which:  # bench.py's C5: the C3-style data in f64, constant optimisation on, 32 populations
        rng = np.random.default_rng(11)
        X = rng.uniform(0.5, 2.0, (5, 100_000)).astype(np.float32)
        y = (X[0] * X[1] * X[2] / (X[3] * X[4] ** 2 + 1)).astype(np.float32)
        opts = Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp", "log"], populations=32,
                       should_optimize_constants=True)
        run("C5 f64 5 features x 100k rows, constant optimisation (32 populations)", X.astype(np.float64),
            y.astype(np.float64), opts, int(os.environ.get("C5_ITERS", "10")))
