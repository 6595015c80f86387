"""TEST INFRASTRUCTURE ONLY — ctypes wrapper of the CPU oracle (``oracle/build/liboracle.so``).

Used by ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg as the
parity checker / CPU baseline.  The product path (``symbolicregression.jl_amd``) never imports it.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(_HERE, "build", "liboracle.so")


def build() -> None:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def _load():
    if not os.path.exists(LIB):
        build()
    lib = ctypes.CDLL(LIB)
    P = ctypes.c_void_p
    I64 = ctypes.c_int64
    I = ctypes.c_int
    D = ctypes.c_double
    lib.oracle_op_id.restype = I
    lib.oracle_op_id.argtypes = [ctypes.c_char_p, I]
    for sfx in ("f32", "f64"):
        f = getattr(lib, f"oracle_eval_tree_{sfx}")
        f.restype = I
        f.argtypes = [I64, P, P, P, P, P, P, I, P, I, P, I64, I64, P, P, I]
        f = getattr(lib, f"oracle_eval_loss_{sfx}")
        f.restype = I
        f.argtypes = [I64, P, P, P, P, P, P, I, P, I, P, I64, I64, P, P, I, D, I, P, P, I]
        f = getattr(lib, f"oracle_eval_loss_batch_{sfx}")
        f.restype = I
        f.argtypes = [I64, P, P, P, P, P, P, P, I, P, I, P, I64, I64, P, P, I, D, I, I, P, P, I]
    return lib


_lib = None


def lib():
    global _lib
    if _lib is None:
        _lib = _load()
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def _ids(names, degree):
    out = []
    for n in names:
        i = lib().oracle_op_id(n.encode(), degree)
        if i == 0:
            raise ValueError(f"oracle has no operator {n!r}")
        out.append(i)
    return np.array(out if out else [0], dtype=np.int32)


class Oracle:
    """CPU restatement of eval_tree_array / _eval_loss for one operator set."""

    def __init__(self, unaops, binops):
        self.unaops = tuple(unaops)
        self.binops = tuple(binops)
        self.un = _ids(self.unaops, 1)
        self.bi = _ids(self.binops, 2)

    @classmethod
    def from_options(cls, options):
        return cls(options.operators.unaops, options.operators.binops)

    @staticmethod
    def _sfx(dtype):
        return "f32" if np.dtype(dtype) == np.float32 else "f64"

    def eval_tree_array(self, tb, k, X, perturb=0):
        """tb: TreeBatch-like (offsets/degree/op/feature/constant/val); X: [nf, n]."""
        X = np.asarray(X)
        dtype = X.dtype
        Xj = np.ascontiguousarray(X.T)
        b, e = int(tb.offsets[k]), int(tb.offsets[k + 1])
        val = np.ascontiguousarray(tb.val[b:e].astype(dtype))
        out = np.empty(X.shape[1], dtype=dtype)
        comp = ctypes.c_int(0)
        f = getattr(lib(), f"oracle_eval_tree_{self._sfx(dtype)}")
        ok = f(e - b, _p(tb.degree[b:e]), _p(tb.op[b:e]), _p(tb.feature[b:e]), _p(tb.constant[b:e]), _p(val),
               _p(self.un), len(self.unaops), _p(self.bi), len(self.binops), _p(Xj), X.shape[0], X.shape[1],
               _p(out), ctypes.byref(comp), int(perturb))
        if not ok:
            raise ValueError("oracle: malformed tree")
        return out, bool(comp.value)

    def eval_loss_batch(self, tb, X, y, w=None, loss_kind=0, accum="f64", n_threads=1, perturb=0, loss_param=0.0):
        X = np.asarray(X)
        dtype = X.dtype
        Xj = np.ascontiguousarray(X.T)
        y = np.ascontiguousarray(y, dtype=dtype)
        w = None if w is None else np.ascontiguousarray(w, dtype=dtype)
        val = np.ascontiguousarray(tb.val.astype(dtype))
        n_trees = len(tb.offsets) - 1
        loss = np.empty(n_trees, dtype=dtype)
        comp = np.empty(n_trees, dtype=np.int32)
        f = getattr(lib(), f"oracle_eval_loss_batch_{self._sfx(dtype)}")
        ok = f(n_trees, _p(np.ascontiguousarray(tb.offsets, dtype=np.int64)), _p(tb.degree), _p(tb.op),
               _p(tb.feature), _p(tb.constant), _p(val), _p(self.un), len(self.unaops), _p(self.bi),
               len(self.binops), _p(Xj), X.shape[0], X.shape[1], _p(y), _p(w), int(loss_kind),
               float(loss_param), 0 if accum == "ref" else 1, int(n_threads), _p(loss), _p(comp), int(perturb))
        if not ok:
            raise ValueError("oracle: malformed tree")
        return loss, comp.astype(bool)

    def loss_grad_fd(self, tb, X, y, w=None, loss_kind=0, rel_step=1e-5, n_threads=8, with_error=False, loss_param=0.0):
        """Central finite differences of the f64 loss with respect to every tree's constants
        (pre-order, get_scalar_constants), the gradient-free objective the reference's Optim BFGS
        differentiates (src/ConstantOptimization.jl:77-116), Richardson-extrapolated over steps h
        and h/2.  Returns (grads, loss, complete) in the layout of ``sr_amd.eval_grad_batch``
        (plus |D(h) - D(h/2)|, a truncation-error estimate, with ``with_error``)."""
        g1, loss0, comp0 = self._fd(tb, X, y, w, loss_kind, rel_step, n_threads, loss_param)
        g2, _, _ = self._fd(tb, X, y, w, loss_kind, rel_step / 2, n_threads, loss_param)
        g = (4 * g2 - g1) / 3
        if with_error:
            return g, loss0, comp0, np.abs(g2 - g1)
        return g, loss0, comp0

    def _fd(self, tb, X, y, w, loss_kind, rel_step, n_threads, loss_param=0.0):
        X = np.asarray(X, dtype=np.float64)
        mask = (tb.degree == 0) & (tb.constant != 0)
        cpos = np.nonzero(mask)[0]
        base_val = tb.val.astype(np.float64)
        loss0, comp0 = self.eval_loss_batch(tb, X, y, w, loss_kind, accum="f64", n_threads=n_threads,
                                            loss_param=loss_param)
        if len(cpos) == 0:
            return np.zeros(0), loss0, comp0
        tree_of = np.searchsorted(tb.offsets, cpos, side="right") - 1
        # one perturbed copy of the owning tree per (constant, sign)
        reps = np.repeat(tree_of, 2)
        starts, ends = tb.offsets[reps], tb.offsets[reps + 1]
        sel = np.concatenate([np.arange(s, e) for s, e in zip(starts, ends)])
        offs = np.concatenate([[0], np.cumsum(ends - starts)])
        val = base_val[sel].copy()
        h = rel_step * np.maximum(1.0, np.abs(base_val[cpos]))
        for i, (p, t) in enumerate(zip(cpos, tree_of)):
            for sgn, k in ((1.0, 2 * i), (-1.0, 2 * i + 1)):
                val[offs[k] + (p - tb.offsets[t])] += sgn * h[i]

        class _B:
            pass

        b = _B()
        b.offsets, b.degree, b.op = offs, tb.degree[sel], tb.op[sel]
        b.feature, b.constant, b.val = tb.feature[sel], tb.constant[sel], val
        lp, _ = self.eval_loss_batch(b, X, y, w, loss_kind, accum="f64", n_threads=n_threads, loss_param=loss_param)
        g = (lp[0::2] - lp[1::2]) / (2 * h)
        return g, loss0, comp0
