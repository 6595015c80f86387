"""TEST HELPER: a numpy interpreter of libsr_amd's compiled programs (csrc/sr_ops.h encoding).

It executes exactly the instruction semantics of the HIP kernel (top-of-stack + operand stack,
combined opcodes, the INFSUB and CHECK bits of arg) on the CPU, so CPU tests can validate the tree COMPILER
(constant folding, check placement, fused-unary detection, Sethi–Ullman ordering) against the
oracle without a GPU.  It is not part of the product and is never used as a fallback.
"""
import ctypes

import numpy as np

from sr_amd import _lib

# SrUnaryOp / SrBinaryOp ids (csrc/sr_ops.h)
U = dict(NEG=1, SQUARE=2, CUBE=3, EXP=4, COS=5, SIN=6, TAN=7, LOG=8, LOG2=9, LOG10=10, LOG1P=11, SQRT=12, ABS=13)
B = dict(ADD=1, SUB=2, MUL=3, DIV=4)
MAX_EXP = {np.float32: np.float32(88.72284), np.float64: 709.7827128933841}


def compile_info(options, tb, n_rows, nfeatures, dtype):
    un = (ctypes.c_char_p * max(1, len(options.operators.unaops)))(*[s.encode() for s in options.operators.unaops])
    bi = (ctypes.c_char_p * max(1, len(options.operators.binops)))(*[s.encode() for s in options.operators.binops])
    nt = tb.n_trees
    lens = np.zeros(nt, dtype=np.int32)
    bad = np.zeros(nt, dtype=np.uint8)
    depth = ctypes.c_int()
    s = tb.to_struct()
    dt = _lib.SR_DTYPE_F32 if dtype == np.float32 else _lib.SR_DTYPE_F64
    cap = int(tb.n_nodes) + 16
    rec = np.dtype([("code", "<u4"), ("arg", "<u4"), ("val", "<f4"), ("pad", "<u4")]) if dtype == np.float32 else \
        np.dtype([("code", "<u4"), ("arg", "<u4"), ("val", "<f8")])
    code = np.zeros(cap, dtype=rec)
    _lib.check(_lib.lib.sr_compile_info(dt, len(options.operators.unaops), un, len(options.operators.binops), bi,
                                        ctypes.byref(s), n_rows, nfeatures, lens.ctypes.data_as(ctypes.c_void_p),
                                        bad.ctypes.data_as(ctypes.c_void_p), ctypes.byref(depth),
                                        code.ctypes.data_as(ctypes.c_void_p), cap))
    offs = np.concatenate([[0], np.cumsum(lens)])
    return code, offs, bad.astype(bool), int(depth.value)


def _unary(uid, x, T):
    with np.errstate(all="ignore"):
        if uid == U["NEG"]:
            return -x
        if uid == U["SQUARE"]:
            return x * x
        if uid == U["CUBE"]:
            return x * x * x
        if uid == U["EXP"]:
            return np.where(x > MAX_EXP[T], T(np.inf), np.exp(x)).astype(T)
        if uid == U["COS"]:
            return np.cos(x)
        if uid == U["SIN"]:
            return np.sin(x)
        if uid == U["LOG"]:
            return np.where(x > 0, np.log(np.where(x > 0, x, T(1))), T(np.nan)).astype(T)
        if uid == U["SQRT"]:
            return np.where(x >= 0, np.sqrt(np.where(x >= 0, x, T(0))), T(np.nan)).astype(T)
        if uid == U["ABS"]:
            return np.abs(x)
    raise NotImplementedError(uid)


def _binary(bid, a, b):
    with np.errstate(all="ignore"):
        if bid == B["ADD"]:
            return a + b
        if bid == B["SUB"]:
            return a - b
        if bid == B["MUL"]:
            return a * b
        if bid == B["DIV"]:
            return a / b
    raise NotImplementedError(bid)


def run_program(code, lo, hi, X, T):
    """Execute one tree's program over all rows; returns (values, complete, check_arrays)."""
    n = X.shape[1]
    tos = np.zeros(n, dtype=T)
    stack = []
    complete = True
    big = T(np.finfo(T).max)
    for pc in range(lo, hi):
        opc = int(code["code"][pc])
        arg = int(code["arg"][pc])
        fidx = arg & ((1 << 28) - 1)  # bit 28: INFSUB, bits 29/30: operand-source tags
        val = T(code["val"][pc])
        if opc <= 3:
            if opc >= 2:
                stack.append(tos)
            tos = X[fidx].astype(T) if opc in (0, 2) else np.full(n, val, dtype=T)
        elif opc < 64:
            v = _unary(opc - 3, tos, T).astype(T)
            if arg & (1 << 28):  # INFSUB: fused unary, non-finite input -> +Inf
                v = np.where(np.isfinite(tos), v, T(np.inf)).astype(T)
            tos = v
        else:
            bid, v = divmod(opc - 64, 6)
            bid += 1
            if v in (0, 1):
                o = stack.pop()
            elif v in (2, 3):
                o = X[fidx].astype(T)
            else:
                o = np.full(n, val, dtype=T)
            a, b = (o, tos) if v in (0, 2, 4) else (tos, o)
            tos = _binary(bid, a, b).astype(T)
        if arg & (1 << 31):  # CHECK: isfinite(sum(array)) (f64 sum)
            s = np.sum(tos.astype(np.float64))
            if not np.isfinite(tos).all() or not abs(s) <= float(big):
                complete = False
    return tos, complete


def eval_loss_batch(options, tb, X, y, dtype=np.float32):
    code, offs, bad, _ = compile_info(options, tb, X.shape[1], X.shape[0], dtype)
    nt = tb.n_trees
    loss = np.empty(nt, dtype=dtype)
    comp = np.zeros(nt, dtype=bool)
    for k in range(nt):
        if bad[k]:
            loss[k] = np.inf
            continue
        v, ok = run_program(code, offs[k], offs[k + 1], X, dtype)
        comp[k] = ok
        with np.errstate(all="ignore"):
            loss[k] = np.mean(((v - y).astype(dtype) ** 2).astype(np.float64)) if ok else np.inf
    return loss, comp
