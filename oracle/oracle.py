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

    def perturb_code(self, name, degree):
        """`perturb` bits that restrict the +-1-ulp conditioning probe to one operator: pass
        `seed | perturb_code(name, degree)` (de_eval_impl.h: perturb_unary / perturb_binary)."""
        return int(_ids([name], degree)[0] + (0 if degree == 1 else 64)) << 8

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

    def eval_loss_batch(self, tb, X, y, w=None, loss_kind=0, accum="ref", n_threads=1, perturb=0, loss_param=0.0):
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


class _Scorer(ctypes.Structure):
    _fields_ = [("X", ctypes.c_void_p), ("nf", ctypes.c_int64), ("n", ctypes.c_int64), ("y", ctypes.c_void_p),
                ("w", ctypes.c_void_p), ("un", ctypes.c_void_p), ("n_un", ctypes.c_int), ("bi", ctypes.c_void_p),
                ("n_bi", ctypes.c_int), ("loss_kind", ctypes.c_int), ("loss_param", ctypes.c_double),
                ("n_threads", ctypes.c_int)]


class SearchScorer:
    """The oracle as the search engine's CPU scorer (C callbacks `oracle_search_loss` /
    `oracle_search_grad` for ``sr_search_use_callbacks``): the same engine, seeds and draws as a
    device-scored search, every scoring call answered on the host cores by this port (loss folded in
    T as the reference does; gradients by central finite differences, as the reference's Optim BFGS
    uses by default).  bench.py's search CPU baseline ("port")."""

    def __init__(self, orc, X, y, w=None, loss_kind=0, loss_param=0.0, n_threads=1):
        X = np.asarray(X)
        dt = X.dtype
        sfx = Oracle._sfx(dt)
        self._keep = [np.ascontiguousarray(X.T), np.ascontiguousarray(y, dtype=dt),
                      None if w is None else np.ascontiguousarray(w, dtype=dt), orc.un, orc.bi]
        Xj, yy, ww = self._keep[:3]
        self.st = _Scorer(_p(Xj), X.shape[0], X.shape[1], _p(yy), _p(ww), _p(orc.un), len(orc.unaops), _p(orc.bi),
                          len(orc.binops), int(loss_kind), float(loss_param), int(n_threads))
        self.user = ctypes.cast(ctypes.pointer(self.st), ctypes.c_void_p)
        L = lib()
        self.loss_addr = ctypes.cast(getattr(L, f"oracle_search_loss_{sfx}"), ctypes.c_void_p).value
        self.grad_addr = ctypes.cast(getattr(L, f"oracle_search_grad_{sfx}"), ctypes.c_void_p).value


def _fwd_unary(name, x, y):
    """d op(x) / dx of the device's derivative rules (csrc/sr_ops.h sr_unary_deriv)."""
    if name == "cos":
        return -np.sin(x)
    if name == "sin":
        return np.cos(x)
    if name == "exp":
        return y
    if name in ("log", "safe_log"):
        return 1.0 / x
    if name in ("sqrt", "safe_sqrt"):
        return 0.5 / y
    if name == "square":
        return 2.0 * x
    if name == "cube":
        return 3.0 * x * x
    if name == "neg":
        return -np.ones_like(x)
    if name == "abs":
        return np.sign(x)
    raise ValueError(f"no forward-mode rule for {name!r}")


_UNARY_FN = {"cos": np.cos, "sin": np.sin, "exp": np.exp, "log": np.log, "safe_log": np.log, "sqrt": np.sqrt,
             "safe_sqrt": np.sqrt, "square": np.square, "cube": lambda x: x * x * x, "neg": np.negative,
             "abs": np.abs}


def loss_grad_forward(orc, tb, X, y, w=None, loss_kind=0):
    """Forward-mode (dual-number) gradient of the Float64 L2 loss with respect to every tree's constants
    (pre-order, get_scalar_constants) — the restatement of the device's forward-mode kernel
    (csrc/sr_grad_impl.h: d loss / d pred = 2(pred - y), times the weight, / n or / Σw) with numpy's
    libm.  Only complete trees are differentiated (zeros otherwise), as the device does.  Returns
    (grads, loss, complete) in the layout of ``sr_amd.eval_grad_batch``."""
    if loss_kind != 0:
        raise ValueError("loss_grad_forward restates L2DistLoss only")
    X = np.asarray(X, dtype=np.float64)
    y = np.asarray(y, dtype=np.float64)
    loss, comp = orc.eval_loss_batch(tb, X, y, w, accum="f64", n_threads=8)
    denom = float(np.sum(w)) if w is not None else float(X.shape[1])
    grads = []
    for k in range(len(tb.offsets) - 1):
        b, e = int(tb.offsets[k]), int(tb.offsets[k + 1])
        deg, op, feat = tb.degree[b:e], tb.op[b:e], tb.feature[b:e]
        con, val = tb.constant[b:e], tb.val[b:e].astype(np.float64)
        cidx = np.cumsum((deg == 0) & (con != 0)) - 1
        nc = int(np.count_nonzero((deg == 0) & (con != 0)))
        if nc == 0:
            continue
        if not comp[k]:
            grads.append(np.zeros(nc))
            continue
        pos = [0]

        def ev():
            i = pos[0]
            pos[0] += 1
            if deg[i] == 0:
                if con[i]:
                    d = np.zeros((nc, X.shape[1]))
                    d[cidx[i]] = 1.0
                    return np.full(X.shape[1], val[i]), d
                return X[int(feat[i]) - 1].copy(), np.zeros((nc, X.shape[1]))
            if deg[i] == 1:
                name = orc.unaops[int(op[i]) - 1]
                xv, dx = ev()
                yv = _UNARY_FN[name](xv)
                return yv, _fwd_unary(name, xv, yv) * dx
            name = orc.binops[int(op[i]) - 1]
            av, da = ev()
            bv, db = ev()
            if name == "+":
                return av + bv, da + db
            if name == "-":
                return av - bv, da - db
            if name == "*":
                return av * bv, bv * da + av * db
            if name == "/":
                r = av / bv
                return r, (1.0 / bv) * da + (-r / bv) * db
            raise ValueError(f"no forward-mode rule for {name!r}")

        pred, dpred = ev()
        coef = 2.0 * (pred - y)
        if w is not None:
            coef = coef * np.asarray(w, dtype=np.float64)
        grads.append(dpred @ coef / denom)
    g = np.concatenate(grads) if grads else np.zeros(0)
    return g, loss, comp
