"""TEST HELPER: comparison utilities shared by the parity tests."""
import numpy as np


def rel(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    both_inf = np.isinf(a) & np.isinf(b) & (np.sign(a) == np.sign(b))
    with np.errstate(invalid="ignore", divide="ignore"):
        return np.where(both_inf, 0.0, np.abs(a - b) / np.maximum(np.abs(b), 1e-30))


PERTURB_SEEDS = (1, 2, 3, 4)
REL_BAR = 1e-4  # north_star: losses within 1e-4 relative (f32)


def loss_tolerance(orc, tb, X, y, w=None, loss_kind=0, loss_param=0.0, rel_bar=REL_BAR, spread_factor=4.0):
    """Per-tree loss tolerance for EVERY tree: max(rel_bar * |loss|, spread_factor * libm spread).

    The oracle evaluates every tree five times: as is, and four times with every libm result (exp,
    cos, log, ...; not the IEEE-exact + - * / sqrt) nudged by one ulp with a pseudo-random sign
    per (node, row) — the independent last-bit differences two libms make (glibc, ROCm OCML and
    Julia's own are each accurate to < 1 ulp, not bitwise equal).  The spread of the four perturbed
    losses around the unperturbed one measures how much a tree amplifies last-bit differences
    (cancellation such as c - log(exp(x)), cos of exp(exp(x)), ...).  Well-conditioned trees get the
    north-star bar itself; an ill-conditioned one gets `spread_factor` times its measured spread —
    no tree is excluded.  Returns (tol, loss, complete, n_widened) of the unperturbed oracle;
    n_widened counts complete trees whose tolerance exceeds the plain bar.
    """
    # (accum "ref": LossFunctions' in-order fold in T, what the device returns since round 6)
    kw = dict(w=w, loss_kind=loss_kind, accum="ref", n_threads=8, loss_param=loss_param)
    l0, c0 = orc.eval_loss_batch(tb, X, y, **kw)
    spread = np.zeros(len(l0))
    for seed in PERTURB_SEEDS:  # one pattern of signs can cancel by chance; four rarely all do
        lp, cp = orc.eval_loss_batch(tb, X, y, perturb=seed, **kw)
        with np.errstate(invalid="ignore"):
            d = np.abs(lp.astype(np.float64) - l0.astype(np.float64))
        # a perturbation that tips a tree over a finiteness edge measures nothing about its loss
        spread = np.maximum(spread, np.where(cp & c0 & np.isfinite(d), d, 0.0))
    base = rel_bar * np.abs(l0.astype(np.float64))
    tol = np.maximum(base, spread_factor * spread)
    n_widened = int(np.sum(c0 & (tol > base)))
    return tol, l0, c0, n_widened


def assert_losses_within(loss, ref_loss, comp, tol, what=""):
    """Every complete tree: |device - oracle| <= tol (per tree), and +Inf exactly where the oracle has
    +Inf (a loss fold that overflows; an Inf oracle loss must not widen the bar to Inf)."""
    loss = np.asarray(loss, dtype=np.float64)
    ref = np.asarray(ref_loss, dtype=np.float64)
    comp = np.asarray(comp, dtype=bool)
    inf_mism = np.nonzero(comp & (np.isinf(loss) != np.isinf(ref)))[0]
    assert len(inf_mism) == 0, (what, "Inf mismatch", [(int(k), float(loss[k]), float(ref[k])) for k in inf_mism[:5]])
    with np.errstate(invalid="ignore"):
        err = np.where(loss == ref, 0.0, np.abs(loss - ref))  # equal infinities (a mean that overflows) agree
    bad = np.nonzero(comp & ~(err <= tol))[0]
    assert len(bad) == 0, (what, [(int(k), float(loss[k]), float(ref[k]), float(tol[k])) for k in bad[:5]])
    return err
