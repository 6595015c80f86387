"""Where a small call's interpreter kernel spends its time: per-wave wall-clock stamps (100 MHz) from a
-DSR_STAMPS build of the library (tools/ab_lib.sh HEAD stamps -DSR_STAMPS; run with
SR_AMD_LIB=ab/stamps/libsr_amd.so).  Points (csrc/sr_tile_impl.h SR_STAMP): 0 entry, 1 prologue
issued, 2 first tile staged, 3 first window consumed, 4 first tile's trees done, 5 all tiles done,
6 results written.  Prints, per configuration, the median / p90 over waves of each point relative to
the kernel's first entry and of each segment, plus the spread of wave entries (dispatch ramp).

usage: SR_AMD_LIB=ab/stamps/libsr_amd.so python tools/stamps.py [config ...]   (c3, c3s, c5, c1, c2s)"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "symbolicregression.jl_amd")]
import numpy as np  # noqa: E402

import sr_amd  # noqa: E402
from sr_amd import Dataset, Options, eval_loss_batch, flatten_trees, gen_random_population  # noqa: E402
from sr_amd import _lib  # noqa: E402

NS = 8
NAMES = ["entry", "prologue", "staged", "window", "tile0", "tiles", "written"]


def stamps(ctx):
    lib = _lib.lib
    f = lib.sr_debug_stamps
    f.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.POINTER(ctypes.c_int64)]
    n = ctypes.c_int64(0)
    f(ctx.handle, None, 0, ctypes.byref(n))
    buf = np.zeros(n.value, dtype=np.uint64)
    f(ctx.handle, buf.ctypes.data, n.value, ctypes.byref(n))
    return buf.reshape(-1, NS).astype(np.int64)


def report(name, st):
    st = st[st[:, 0] > 0]
    t0 = st[:, 0].min()
    rel = (st - t0) * 10.0 / 1000.0  # us
    print(f"== {name}: {len(st)} waves; kernel span {rel[:, 6].max():.2f} us (last result written)")
    for k, nm in enumerate(NAMES):
        v = rel[:, k][st[:, k] > 0]
        if len(v):
            print(f"  t[{nm:8s}] median {np.median(v):7.2f}  p10 {np.quantile(v, .1):7.2f}  p90 {np.quantile(v, .9):7.2f}  max {v.max():7.2f} us")
    for k in range(1, 7):
        ok = (st[:, k] > 0) & (st[:, k - 1] > 0)
        d = (st[ok, k] - st[ok, k - 1]) * 10.0 / 1000.0
        if len(d):
            print(f"  {NAMES[k - 1]:>8s} -> {NAMES[k]:8s} median {np.median(d):7.2f}  p90 {np.quantile(d, .9):7.2f} us")


def main():
    ctx = sr_amd.get_context()
    which = sys.argv[1:] or ["c3", "c1"]
    for cfg in which:
        if cfg == "c3":  # the C3 search's calls: 31 trees x 100k rows f32
            dt, n_rows, n_trees, nf = np.float32, 100_000, 31, 5
        elif cfg == "c1":  # C1: 20 trees x 100 rows f64
            dt, n_rows, n_trees, nf = np.float64, 100, 20, 2
        elif cfg == "c3s":  # the C3 search's average call: 9 trees x 100k rows f32
            dt, n_rows, n_trees, nf = np.float32, 100_000, 9, 5
        elif cfg == "c5":  # the C5 search's average call: 8 trees x 100k rows f64
            dt, n_rows, n_trees, nf = np.float64, 100_000, 8, 5
        else:  # c2s: 1000 trees x 2^20 rows f32
            dt, n_rows, n_trees, nf = np.float32, 1 << 20, 1000, 5
        rng = np.random.default_rng(0)
        X = rng.uniform(0.5, 2.0, (nf, n_rows)).astype(dt)
        y = (X[0] * X[-1] + 1).astype(dt)
        ds = Dataset(X, y)
        opts = Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp", "log"])
        tb = flatten_trees(gen_random_population(n_trees, opts, nf, max_size=20, seed=3), dt)
        for _ in range(20):
            eval_loss_batch(tb, ds, opts)
        report(f"{cfg} ({n_trees} trees x {n_rows} rows {np.dtype(dt).name})", stamps(ctx))


if __name__ == "__main__":
    main()
