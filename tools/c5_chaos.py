"""CPU experiment (no GPU): how sensitive is a Float64 search with BFGS constant optimisation to the
last bits of its scores?  The same seeded search (C3 target in Float64, 4 islands, constant optimisation
p = 0.5) is scored by the oracle (C loss + forward-mode gradient restatement) exactly, and again with
every loss and gradient multiplied by (1 + eps * h), h in [-1, 1) a hash of the value's bits (a
deterministic function of the value, like a second correct scorer's rounding: equal trees keep equal
scores).  Prints how many members differ.  Result: profiles/r03_c5_chaos.txt."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "symbolicregression.jl_amd"), os.path.join(ROOT, "oracle")]
import numpy as np  # noqa: E402

from oracle import Oracle, loss_grad_forward  # noqa: E402
from sr_amd import Options, equation_search, string_tree  # noqa: E402


def hnoise(v, seed):
    b = np.ascontiguousarray(v, dtype=np.float64).view(np.uint64)
    h = (b * np.uint64(0x9E3779B97F4A7C15) + np.uint64(seed)) >> np.uint64(40)
    return (h.astype(np.float64) / 2 ** 24 - 0.5) * 2


def run(X, y, opts, eps_loss, eps_grad, seed, niterations):
    orc = Oracle.from_options(opts)

    def lossf(tb, rows):
        Xv, yv = (X, y) if rows is None else (X[:, rows], y[rows])
        l, c = orc.eval_loss_batch(tb, Xv, yv, accum="f64", n_threads=8)
        l = np.where(c, l, np.inf)
        return l * (1 + eps_loss * hnoise(l, seed))

    def gradf(tb, rows):
        Xv, yv = (X, y) if rows is None else (X[:, rows], y[rows])
        g, l, c = loss_grad_forward(orc, tb, Xv, yv)
        l = np.where(c, l, np.inf) * (1 + eps_loss * hnoise(l, seed))
        return l, g * (1 + eps_grad * hnoise(g, seed))

    r = equation_search(X, y, niterations=niterations, options=opts, seed=5, _loss_fn=lossf, _grad_fn=gradf)
    return r.device_calls, [[string_tree(m.tree, opts.operators) for m in p] for p in r.populations]


def main():
    rng = np.random.default_rng(11)
    X = rng.uniform(0.5, 2.0, (5, 1000))
    y = X[0] * X[1] * X[2] / (X[3] * X[4] ** 2 + 1)
    print("# C5-style search (Float64, 4 islands x 20, BFGS p = 0.5), oracle-scored; perturbation eps * h(bits)")
    print("# ncycles iterations eps_loss eps_grad seed  calls(exact) calls(perturbed)  members_differing/80")
    for nc, it in ((1, 1), (10, 1), (10, 2)):
        opts = Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp", "log"], populations=4,
                       population_size=20, ncycles_per_iteration=nc, maxsize=20, should_optimize_constants=True,
                       optimizer_probability=0.5)
        base = run(X, y, opts, 0.0, 0.0, 0, it)
        again = run(X, y, opts, 0.0, 0.0, 0, it)
        assert again == base  # the exact run is deterministic
        for el, eg, seed in ((2e-16, 0.0, 1), (0.0, 2e-16, 1), (2e-16, 2e-16, 2)):
            r = run(X, y, opts, el, eg, seed, it)
            diff = sum(a != b for pa, pb in zip(base[1], r[1]) for a, b in zip(pa, pb))
            print(f"{nc:8d} {it:10d} {el:8.0e} {eg:8.0e} {seed:4d}  {base[0]:12d} {r[0]:16d}  {diff:8d}")


if __name__ == "__main__":
    main()
