"""Host compile time vs batch size and SR_AMD_COMPILE_THREADS, wall and process CPU time, plus the
pool threads' state (does the compile pool run pieces in parallel?)."""
import ctypes, os, sys, time
sys.path[:0] = [os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "symbolicregression.jl_amd")]
import numpy as np
from sr_amd import Options, flatten_trees, gen_random_population, _lib
opts = Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp", "log"])
pop = gen_random_population(10000, opts, 5, seed=1)
un = (ctypes.c_char_p * 3)(*[s.encode() for s in opts.operators.unaops])
bi = (ctypes.c_char_p * 4)(*[s.encode() for s in opts.operators.binops])
for nt in (100, 1000, 10000):
    tb = flatten_trees(pop[:nt], np.float32)
    lens = np.zeros(nt, dtype=np.int32); bad = np.zeros(nt, dtype=np.uint8); depth = ctypes.c_int()
    s = tb.to_struct(); ts = []; cs = []
    for _ in range(20):
        t0 = time.perf_counter(); c0 = time.process_time()
        _lib.check(_lib.lib.sr_compile_info(_lib.SR_DTYPE_F32, 3, un, 4, bi, ctypes.byref(s), 1 << 20, 5,
            lens.ctypes.data_as(ctypes.c_void_p), bad.ctypes.data_as(ctypes.c_void_p), ctypes.byref(depth), None, 0))
        ts.append(time.perf_counter() - t0); cs.append(time.process_time() - c0)
    print(os.environ.get("SR_AMD_COMPILE_THREADS"), nt, f"{np.min(ts)*1e3:.3f} ms min, {np.median(ts)*1e3:.3f} med", f"cpu {np.median(cs)*1e3:.3f} ms", flush=True)
print(open("/proc/self/status").read().split("Threads:")[1].split()[0], "threads")
import subprocess
out = subprocess.run(["ps", "-L", "-o", "tid,stat,pcpu,psr,wchan:20", "-p", str(os.getpid())], capture_output=True, text=True).stdout
print(out)
for tid in sorted(int(t) for t in os.listdir("/proc/self/task")):
    print(tid, sorted(os.sched_getaffinity(tid)))
