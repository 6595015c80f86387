"""Gradient-kernel A/B: bench.grad_roofline_batch on the C5 search's final members and on
a fixed synthetic population (2,000 random trees with constants, C5's data), per tuning setting given as
name=value[,name=value] arguments (alternating passes).  One JSON line per (population, setting, pass)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "symbolicregression.jl_amd"), ROOT, os.path.join(ROOT, "tools")]
import numpy as np  # noqa: E402


def main():
    import bench
    import sr_amd
    from c5_grad_profile import c5_setup
    from sr_amd import equation_search, flatten_trees, gen_random_population

    X, y, o = c5_setup()
    res = equation_search(X, y, niterations=int(os.environ.get("C5_ITERS", "20")), options=o, seed=0)
    pops = {"c5_members": flatten_trees([m.tree for p in res.populations for m in p if m.tree.count_constants() > 0],
                                        np.float64)}
    syn = [t for t in gen_random_population(4000, o, 5, max_size=20, dtype=np.float64, seed=7) if t.count_constants() > 0]
    pops["synthetic"] = flatten_trees(syn[:2000], np.float64)
    ctx = sr_amd.get_context()
    settings = [dict(kv.split("=") for kv in a.split(",")) for a in sys.argv[1:]] or [{}]
    for pas in range(2):
        for st in settings:
            for k, v in st.items():
                ctx.set_tuning(k, int(v))
            for name, tb in pops.items():
                r = bench.grad_roofline_batch(tb, X, y, o)
                print(json.dumps({"pop": name, "setting": st, "pass": pas, "frac": r["frac"],
                                  "kernel_ms": r["kernel_ms_per_call"], "trees": r["trees"],
                                  "buckets": [(b["kt"], b["items"], round(b["kernel_ms"], 4), round(b["frac"], 4))
                                              for b in r["buckets"]]}), flush=True)


if __name__ == "__main__":
    main()
