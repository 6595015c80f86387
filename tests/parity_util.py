"""TEST HELPER: comparison utilities shared by the parity tests."""
import numpy as np


def rel(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    both_inf = np.isinf(a) & np.isinf(b) & (np.sign(a) == np.sign(b))
    with np.errstate(invalid="ignore", divide="ignore"):
        return np.where(both_inf, 0.0, np.abs(a - b) / np.maximum(np.abs(b), 1e-30))


def well_conditioned(orc, tb, X, y, w=None, loss_kind=0, tol=1e-5):
    """Trees whose Float32 loss is determined by the data, not by rounding.

    The f32 loss of the oracle is compared with the same tree evaluated in f64 (constants and data
    widened exactly).  Where they differ by more than `tol`, the f32 result is dominated by
    rounding amplified through the tree (e.g. cos of exp(exp(x))): two correctly-rounded libms
    (glibc, ROCm OCML, Julia's own) legitimately disagree there, so the 1e-4 loss bar of the
    north star applies to the well-conditioned trees only; flags are compared on every tree.
    Returns (mask, o32_loss, o32_complete).
    """
    l32, c32 = orc.eval_loss_batch(tb, X, y, w=w, loss_kind=loss_kind, accum="f64", n_threads=8)
    X64 = np.asarray(X, dtype=np.float64)
    y64 = np.asarray(y, dtype=np.float64)
    w64 = None if w is None else np.asarray(w, dtype=np.float64)
    l64, c64 = orc.eval_loss_batch(tb.astype(np.float64), X64, y64, w=w64, loss_kind=loss_kind, accum="f64",
                                   n_threads=8)
    mask = c32 & c64 & (rel(l32, l64) < tol)
    return mask, l32, c32
