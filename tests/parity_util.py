"""TEST HELPER: comparison utilities shared by the parity tests."""
import numpy as np


def rel(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    both_inf = np.isinf(a) & np.isinf(b) & (np.sign(a) == np.sign(b))
    with np.errstate(invalid="ignore", divide="ignore"):
        return np.where(both_inf, 0.0, np.abs(a - b) / np.maximum(np.abs(b), 1e-30))


PERTURB_SEEDS = (1, 2, 3, 4)


def well_conditioned(orc, tb, X, y, w=None, loss_kind=0, tol=2e-5, loss_param=0.0):
    """Trees whose loss is determined by the data, not by how the libm rounds.

    The oracle evaluates every tree five times: as is, and four times with every libm result (exp,
    cos, log, ...; not the IEEE-exact + - * / sqrt) nudged by one ulp with a pseudo-random sign
    per (node, row) — the independent last-bit differences two libms make.  Where the loss moves
    by more than `tol`, the tree amplifies last-bit differences (cancellation such as
    c - log(exp(x)), cos of exp(exp(x)), ...): two correctly rounded libms (glibc, ROCm OCML,
    Julia's own) legitimately disagree there, and so would the reference itself.  The north-star
    loss bar (1e-4 relative) is applied to the well-conditioned trees; `complete` flags are
    compared on every tree.  Returns (mask, loss, complete) of the unperturbed oracle.
    """
    kw = dict(w=w, loss_kind=loss_kind, accum="f64", n_threads=8, loss_param=loss_param)
    l0, c0 = orc.eval_loss_batch(tb, X, y, **kw)
    mask = c0.copy()
    for seed in PERTURB_SEEDS:  # one pattern of signs can cancel by chance; four rarely all do
        lp, cp = orc.eval_loss_batch(tb, X, y, perturb=seed, **kw)
        mask &= cp & (rel(lp, l0) < tol)
    return mask, l0, c0
