"""Host compile latency of small batches (the search's calls: tens to hundreds of trees) through
sr_compile_info (no device).  usage: SR_AMD_LIB=... python tools/compile_small_bench.py"""
import ctypes, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "symbolicregression.jl_amd")]
import numpy as np
from sr_amd import Options, flatten_trees, gen_random_population, _lib

opts = Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp", "log"])
un = (ctypes.c_char_p * 3)(*[s.encode() for s in opts.operators.unaops])
bi = (ctypes.c_char_p * 4)(*[s.encode() for s in opts.operators.binops])
for nt in (20, 40, 100, 280, 1000, 10000):
    tb = flatten_trees(gen_random_population(nt, opts, 5, max_size=20, seed=1), np.float64)
    lens = np.zeros(nt, dtype=np.int32)
    bad = np.zeros(nt, dtype=np.uint8)
    depth = ctypes.c_int()
    s = tb.to_struct()
    ts = []
    for _ in range(200 if nt < 10000 else 10):
        t0 = time.perf_counter()
        _lib.check(_lib.lib.sr_compile_info(_lib.SR_DTYPE_F64, 3, un, 4, bi, ctypes.byref(s), 100, 5,
                                            lens.ctypes.data_as(ctypes.c_void_p), bad.ctypes.data_as(ctypes.c_void_p),
                                            ctypes.byref(depth), None, 0))
        ts.append(time.perf_counter() - t0)
        time.sleep(0.0002)  # (workers go back to sleep between calls, as in a search)
    print(f"trees={nt:6d} median={np.median(ts) * 1e6:9.1f} us  p90={np.quantile(ts, .9) * 1e6:9.1f} us", flush=True)
