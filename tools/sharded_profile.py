"""GPU box: where the row-sharded step's time goes (world size 1, gloo rendezvous, library RCCL)."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "symbolicregression.jl_amd")]
import numpy as np
import torch.distributed as dist
import bench
import sr_amd
from sr_amd import Dataset, Options, _lib, flatten_trees, gen_random_population
from sr_amd.distributed import (finalize, gpu_jsum, gpu_max_checks, gpu_partials_allreduce, init_device_comm,
                                jsum_finite, unpack_flags)
dist.init_process_group("gloo", init_method="tcp://127.0.0.1:29555", rank=0, world_size=1)
ctx = sr_amd.get_context(0)
init_device_comm(ctx=ctx)
opts = Options(**bench.C2_OPS)
tb = flatten_trees(gen_random_population(10000, opts, 5, max_size=30, seed=1), np.float32)
X, y = bench.c2_data(1 << 20, 0)
ds = Dataset(X, y); ds.device_handle(ctx)
n = X.shape[1]
for it in range(4):
    t = [time.perf_counter()]
    packed = gpu_partials_allreduce(tb, ds, opts, n); t.append(time.perf_counter())
    sums, flags = unpack_flags(packed); t.append(time.perf_counter())
    big = np.nonzero(((flags & (_lib.SR_FLAG_NONFINITE | _lib.SR_FLAG_STATIC)) == 0) & ((flags & _lib.SR_FLAG_BIG) != 0))[0]
    sub = tb.take(big)
    mc = gpu_max_checks(sub, opts); t.append(time.perf_counter())
    mine = gpu_jsum(sub, ds, opts, np.arange(big.size), mc, 0, n); t.append(time.perf_counter())
    fin = jsum_finite(np.float32, n, np.array([0, n]), [mine.reshape(big.size * mc, -1)]); t.append(time.perf_counter())
    ok = fin.reshape(big.size, mc).all(axis=1).astype(np.uint8)
    loss, comp = finalize(np.float32, sums, flags, float(n), big, ok); t.append(time.perf_counter())
    print("ms: allreduce-step %.2f unpack %.2f max_checks %.2f jsum %.2f jsum_finite %.2f finalize %.2f  (big=%d mc=%d)" % tuple(
        [1e3 * (b - a) for a, b in zip(t, t[1:])] + [big.size, mc]), flush=True)
dist.destroy_process_group()
