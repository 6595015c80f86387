"""Kernel-time breakdown by operator mix (GPU box).  Prints one line per population."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# SR_AMD_PKG=ab/<name>: another revision's package + library (tools/ab_lib.sh)
sys.path[:0] = [os.path.join(ROOT, os.environ["SR_AMD_PKG"]) if os.environ.get("SR_AMD_PKG")
                else os.path.join(ROOT, "symbolicregression.jl_amd")]
import numpy as np
import hashlib  # noqa: E402

import sr_amd
from sr_amd import Options, Dataset, flatten_trees, gen_random_population, eval_loss_batch

n = 1 << 20
DT = np.float64 if os.environ.get("MB_DTYPE", "f32") == "f64" else np.float32
rng = np.random.default_rng(2)
X = rng.standard_normal((5, n)).astype(DT)
y = (2 * np.cos(X[3]) + X[0] ** 2 - 2).astype(DT)
ds = Dataset(X, y)
ctx = sr_amd.get_context()
mixes = {
    "arith(+-*/)": dict(binary_operators=["+", "-", "*"], unary_operators=["neg"]),
    "arith+div": dict(binary_operators=["+", "-", "*", "/"], unary_operators=["neg"]),
    "C2(+-*/ cos exp log)": dict(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp", "log"]),
    "cos-only": dict(binary_operators=["+", "*"], unary_operators=["cos"]),
    "exp-only": dict(binary_operators=["+", "*"], unary_operators=["exp"]),
    "sin-only": dict(binary_operators=["+", "*"], unary_operators=["sin"]),
    "log-only": dict(binary_operators=["+", "*"], unary_operators=["log"]),
    "C2-complete": "C2(+-*/ cos exp log)",
    "C2-dead": "C2(+-*/ cos exp log)",
}
only = sys.argv[1:]  # optional: mix names to run (profiling one population at a time)
for name, kw in mixes.items():
    if only and not any(name.startswith(o) for o in only):
        continue
    if isinstance(kw, str):  # a subset of another population: its complete or its dead trees
        opts = Options(**mixes[kw])
        full = gen_random_population(10000, opts, 5, seed=1)
        _, c0 = eval_loss_batch(flatten_trees(full, DT), ds, opts)
        keep = c0 if name.endswith("complete") else ~c0
        tb = flatten_trees([t for t, k in zip(full, keep) if k], DT)
    else:
        opts = Options(**kw)
        tb = flatten_trees(gen_random_population(10000, opts, 5, seed=1), DT)
    eval_loss_batch(tb, ds, opts)
    ks, ts, ph = [], [], []
    for _ in range(5):
        t0 = time.perf_counter()
        l, c = eval_loss_batch(tb, ds, opts)
        ts.append(time.perf_counter() - t0)
        ks.append(ctx.last_kernel_ms()[0])
        ph.append(ctx.last_phase_ms())
    k = float(np.median(ks)); t = float(np.median(ts)) * 1e3
    ne = tb.n_nodes * n
    print(f"{name:24s} nodes={tb.n_nodes:7d} ops={tb.n_operator_nodes:6d} complete={c.mean():.3f} "
          f"kernel={k:7.3f}ms step={t:7.3f}ms  {ne / k / 1e9:8.1f} Gnode/s(kernel)  {ne / t / 1e9:8.1f} Gnode/s(step)"
          f"  phases(compile/launch/wait/exact/final)=" + "/".join(f"{v:.2f}" for v in np.median(np.array(ph), 0))
          + f"  derived={ctx.last_derived_columns()} exact_trees={ctx.last_exact_trees()}"
          f" exact_kernel={ctx.last_exact_kernel_ms():.3f}ms"
          f"  results={hashlib.sha1(np.ascontiguousarray(l).tobytes() + np.ascontiguousarray(c).tobytes()).hexdigest()[:12]}",
          flush=True)
