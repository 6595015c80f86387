"""Diagnostic: full-view flags (register-stack and LDS-stack kernels) vs row-sharded exact path vs oracle."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "symbolicregression.jl_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import numpy as np
import sr_amd
from sr_amd import Dataset, Options, eval_loss_batch, flatten_trees, gen_random_population, parse_expression, _lib
from sr_amd.distributed import finalize, gpu_jsum, gpu_max_checks, gpu_partials_packed, jsum_finite, unpack_flags
from oracle import Oracle
from test_jsum import cases

opts = Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp", "log"])
n = 9000
rng = np.random.default_rng(91)
X = rng.standard_normal((5, n)).astype(np.float32)
y = (2 * np.cos(X[3]) + X[0] ** 2 - 2).astype(np.float32)
X[2] = np.resize(cases()["mixed_overflow_pairwise"], n)
X[4, :4000] = 3e38 / 4000 * 1.3
trees = gen_random_population(600, opts, 5, seed=91)
trees += [parse_expression(e, opts) for e in ("x3 * 1.0", "x3 + x1", "x5 * 1.0", "(x5 * 0.5) + (x1 * 1.0)")]
tb = flatten_trees(trees, np.float32)
res = {}
for R in ("0", "8"):
    ctx = sr_amd.device.DeviceContext(0) if R == "8" else sr_amd.get_context()
    if R == "8":
        os.environ["SR_AMD_ROWS_PER_LANE"] = "8"
        ctx.close(); ctx = sr_amd.device.DeviceContext(0)
    d = Dataset(X, y)
    res[R] = eval_loss_batch(tb, d, opts, ctx=ctx)[1]
    d.free_device()
os.environ.pop("SR_AMD_ROWS_PER_LANE")
cut = 4321
shards = [Dataset(np.ascontiguousarray(X[:, :cut]), np.ascontiguousarray(y[:cut])),
          Dataset(np.ascontiguousarray(X[:, cut:]), np.ascontiguousarray(y[cut:]))]
packed = sum(gpu_partials_packed(tb, sh, opts, n) for sh in shards)
sums, flags = unpack_flags(packed)
big = np.nonzero(((flags & 5) == 0) & ((flags & 2) != 0))[0]
mc = gpu_max_checks(tb, opts)
folds = [gpu_jsum(tb, sh, opts, big, mc, off, n) for sh, off in zip(shards, (0, cut))]
fin = jsum_finite(np.float32, n, [0, cut, n], [f.reshape(big.size * mc, -1) for f in folds])
ok = fin.reshape(big.size, mc).all(axis=1)
_, comp = finalize(np.float32, sums, flags, float(n), big, ok)
_, oc = Oracle.from_options(opts).eval_loss_batch(tb, X, y, n_threads=8)
print("big:", big.tolist())
for k in range(tb.n_trees):
    row = (bool(res["0"][k]), bool(res["8"][k]), bool(comp[k]), bool(oc[k]))
    if len(set(row)) > 1:
        print(k, "vstk/lds/shard/oracle", row, "flags", int(flags[k]), sr_amd.string_tree(tb.tree(k), opts.operators))
print("done")
