"""TEST HELPER: a numpy interpreter of libsr_amd's compiled programs (csrc/sr_ops.h encoding).

It executes exactly the instruction semantics of the HIP kernel (top-of-stack + statically
assigned operand-stack slots, combined opcodes, the push field and CHECK bit of the meta word) on
the CPU, so CPU tests can validate the tree COMPILER
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
    rec = np.dtype([("op", "<u4"), ("meta", "<u4"), ("val", "<f4"), ("c1", "<u4")]) if dtype == np.float32 else \
        np.dtype([("op", "<u4"), ("meta", "<u4"), ("val", "<f8")], align=False)
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


# opcode ranges and meta fields (csrc/sr_ops.h)
LOAD_FEAT, LOAD_CONST, LOAD_FEAT_PUSH, LOAD_CONST_PUSH = 0, 1, 2, 3
UNARY0, UNARY_INF0, BINARY0, PAIR0 = 4, 40, 80, 256
CHECK = 1 << 31
OP_MASK, POST_SHIFT, POST_INF, POST_CHECK = 0x1FF, 16, 1 << 22, 1 << 23
PBC_SHIFT, PBC_CHECK = 24, 1 << 27  # post binary with a constant: 1 +c, 2 -c, 3 c-, 4 *c, 5 /c, 6 c/


def operand(meta):
    return int(meta) & 0xFFFF


def push_slot(meta):
    return ((int(meta) >> 24) & 0x3F) - 1


def is_check(meta):
    return (int(meta) >> 31) & 1


def is_infsub(op):
    return UNARY_INF0 <= int(op) < BINARY0


def run_program(code, lo, hi, X, T):
    """Execute one tree's program over all rows; returns (values, complete)."""
    n = X.shape[1]
    tos = np.zeros(n, dtype=T)
    slots = {}
    complete = True
    big = T(np.finfo(T).max)
    def checked(v):  # isfinite(sum(array)) (f64 sum)
        s = np.sum(v.astype(np.float64))
        return np.isfinite(v).all() and abs(s) <= float(big)

    for pc in range(lo, hi):
        word = int(code["op"][pc])
        opc = word & OP_MASK
        meta = int(code["meta"][pc])
        val = T(code["val"][pc])
        if opc < UNARY0:  # LOAD_FEAT / LOAD_CONST, the _PUSH forms storing the old tos first
            if opc >= LOAD_FEAT_PUSH:
                assert push_slot(meta) >= 0
                slots[push_slot(meta)] = tos
            else:
                assert push_slot(meta) < 0
            tos = X[operand(meta)].astype(T) if opc in (LOAD_FEAT, LOAD_FEAT_PUSH) else np.full(n, val, dtype=T)
        elif opc < BINARY0:
            inf = is_infsub(opc)
            v = _unary(opc - (UNARY_INF0 if inf else UNARY0), tos, T).astype(T)
            if inf:  # fused unary: non-finite input -> +Inf
                v = np.where(np.isfinite(tos), v, T(np.inf)).astype(T)
            tos = v
        elif opc >= PAIR0:  # op(leaf, leaf): FF / FC / CF (+3: push the old tos first)
            bid, v = divmod(opc - PAIR0, 6)
            bid += 1
            if v >= 3:
                slots[push_slot(meta)] = tos
                v -= 3
            xf = X[operand(meta)].astype(T)
            if v == 0:
                o = X[int(code["val"][pc].view(np.uint32) if T == np.float32 else
                          np.array([code["val"][pc]]).view(np.uint64)[0] & 0xFFFFFFFF)].astype(T)
                a, b = xf, o
            elif v == 1:
                a, b = xf, np.full(n, val, dtype=T)
            else:
                a, b = np.full(n, val, dtype=T), xf
            tos = _binary(bid, a, b).astype(T)
        else:
            bid, v = divmod(opc - BINARY0, 6)
            bid += 1
            if v in (0, 1):
                o = slots.pop(operand(meta))
            elif v in (2, 3):
                o = X[operand(meta)].astype(T)
            else:
                o = np.full(n, val, dtype=T)
            a, b = (o, tos) if v in (0, 2, 4) else (tos, o)
            tos = _binary(bid, a, b).astype(T)
        if is_check(meta) and not checked(tos):
            complete = False
        post = (word >> POST_SHIFT) & 0x3F  # a unary node fused into this instruction
        if post:
            v = _unary(post, tos, T).astype(T)
            if word & POST_INF:  # fused form: non-finite input -> +Inf
                v = np.where(np.isfinite(tos), v, T(np.inf)).astype(T)
            tos = v
            if (word & POST_CHECK) and not checked(tos):
                complete = False
        pbc = (word >> PBC_SHIFT) & 7  # then a binary node with a constant operand
        if pbc:
            c = np.full(n, val, dtype=T)
            bid, a, b = {1: (B["ADD"], tos, c), 2: (B["SUB"], tos, c), 3: (B["SUB"], c, tos), 4: (B["MUL"], tos, c),
                         5: (B["DIV"], tos, c), 6: (B["DIV"], c, tos)}[pbc]
            tos = _binary(bid, a, b).astype(T)
            if (word & PBC_CHECK) and not checked(tos):
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
