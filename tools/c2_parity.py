"""GPU diagnostic: the C2 population at full size (10k trees x 2^20 rows) on the device vs the C oracle,
under each launch knob (derived columns, dead-tree probe, LDS code cache), worst trees printed.
usage: python tools/c2_parity.py [n_trees_sample]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "symbolicregression.jl_amd"), os.path.join(ROOT, "oracle"), ROOT]
import numpy as np  # noqa: E402

import sr_amd  # noqa: E402
from bench import C2_OPS, c2_data  # noqa: E402
from oracle import Oracle  # noqa: E402
from sr_amd import Dataset, Options, eval_loss_batch, flatten_trees, gen_random_population, string_tree  # noqa: E402


def main():
    n_sample = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000
    opts = Options(**C2_OPS)
    trees = gen_random_population(10_000, opts, 5, max_size=30, seed=1)
    tb = flatten_trees(trees, np.float32)
    X, y = c2_data(1 << 20, 0)
    ds = Dataset(X, y)
    ctx = sr_amd.get_context()
    variants = {}
    for name, knobs in (("default", {}), ("derived=0", {"derived": 0}), ("probe=0", {"probe": 0}),
                        ("code_cache=0", {"code_cache": 0})):
        for k, v in knobs.items():
            ctx.set_tuning(k, v)
        variants[name] = eval_loss_batch(tb, ds, opts)
        print(name, "derived cols", ctx.last_derived_columns(), "exact", ctx.last_exact_trees(), flush=True)
        for k in knobs:
            ctx.set_tuning(k, {"derived": 1, "probe": 2, "code_cache": 1}[k])
    idx = np.arange(min(n_sample, tb.n_trees))
    sub = tb.take(idx)
    orc = Oracle.from_options(opts)
    t = time.time()
    lf, cf = orc.eval_loss_batch(sub, X, y, accum="f64", n_threads=16)
    lr, cr = orc.eval_loss_batch(sub, X, y, accum="ref", n_threads=16)
    print(f"oracle {time.time() - t:.1f} s", flush=True)
    for name, (l, c) in variants.items():
        l, c = l[idx].astype(np.float64), c[idx]
        with np.errstate(invalid="ignore", divide="ignore"):
            r = np.where(l == lf, 0.0, np.abs(l - lf) / np.abs(lf))
        ok = c & cf
        print(f"{name:14s} flags_equal={np.array_equal(c, cf)} mism={int(np.sum(c != cf))} complete={int(ok.sum())} "
              f"n>1e-4={int(np.sum(r[ok] > 1e-4))} n>1e-6={int(np.sum(r[ok] > 1e-6))} max={np.max(r[ok]):.3e}")
    l, c = variants["default"]
    l = l[idx].astype(np.float64)
    with np.errstate(invalid="ignore", divide="ignore"):
        r = np.where(l == lf, 0.0, np.abs(l - lf) / np.abs(lf))
    r[~(c[idx] & cf)] = 0
    for k in np.argsort(-r)[:15]:
        print(f"tree {k:5d} rel {r[k]:.3e} dev {l[k]:.9g} f64 {lf[k]:.9g} ref {lr[k]:.9g} "
              f"derived0 {variants['derived=0'][0][k]:.9g} probe0 {variants['probe=0'][0][k]:.9g}  "
              f"{string_tree(tb.tree(int(k)), opts.operators)[:160]}")
    with np.errstate(invalid="ignore", divide="ignore"):
        rr = np.abs(lr.astype(np.float64) - lf) / np.abs(lf)
    ok = cf & cr
    print("reference sequential f32 fold vs f64 fold over 2^20 rows: median rel", float(np.median(rr[ok])),
          "p95", float(np.quantile(rr[ok], 0.95)), "max", float(np.max(rr[ok])))


if __name__ == "__main__":
    main()
