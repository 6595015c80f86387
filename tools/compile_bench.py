"""Host compile time of the C2 population (10k trees) through sr_compile_info (GPU box or CPU).
usage: SR_AMD_COMPILE_THREADS=N python tools/compile_bench.py"""
import ctypes, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "symbolicregression.jl_amd")]
import numpy as np
from sr_amd import Options, flatten_trees, gen_random_population, _lib

opts = Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp", "log"])
tb = flatten_trees(gen_random_population(10000, opts, 5, seed=1), np.float32)
un = (ctypes.c_char_p * 3)(*[s.encode() for s in opts.operators.unaops])
bi = (ctypes.c_char_p * 4)(*[s.encode() for s in opts.operators.binops])
lens = np.zeros(tb.n_trees, dtype=np.int32)
bad = np.zeros(tb.n_trees, dtype=np.uint8)
depth = ctypes.c_int()
s = tb.to_struct()
ts = []
for _ in range(20):
    t0 = time.perf_counter()
    _lib.check(_lib.lib.sr_compile_info(_lib.SR_DTYPE_F32, 3, un, 4, bi, ctypes.byref(s), 1 << 20, 5,
                                        lens.ctypes.data_as(ctypes.c_void_p), bad.ctypes.data_as(ctypes.c_void_p),
                                        ctypes.byref(depth), None, 0))
    ts.append(time.perf_counter() - t0)
print(f"threads={os.environ.get('SR_AMD_COMPILE_THREADS', 'default')} nodes={tb.n_nodes} "
      f"median={np.median(ts) * 1e3:.3f} ms min={np.min(ts) * 1e3:.3f} ms cpus={len(os.sched_getaffinity(0))}", flush=True)
