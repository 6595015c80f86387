"""Per-process device context: one ``sr_ctx`` per GPU (one process per GPU; LOCAL_RANK picks it)."""
from __future__ import annotations

import ctypes
import os
import threading

from . import _lib

_lock = threading.Lock()
_contexts: dict = {}
_lane_contexts: dict = {}


class DeviceContext:
    def __init__(self, device: int):
        self.device = device
        h = ctypes.c_void_p()
        _lib.check(_lib.lib.sr_init(device, ctypes.byref(h)))
        self.handle = h
        self._opsets: dict = {}
        self.has_comm = False  # RCCL communicator created (sr_amd.distributed.init_device_comm)

    def opset_id(self, operators) -> int:
        key = operators.key()
        oid = self._opsets.get(key)
        if oid is None:
            un = (ctypes.c_char_p * max(1, len(operators.unaops)))(*[s.encode() for s in operators.unaops])
            bi = (ctypes.c_char_p * max(1, len(operators.binops)))(*[s.encode() for s in operators.binops])
            out = ctypes.c_int()
            _lib.check(
                _lib.lib.sr_register_opset(
                    self.handle, len(operators.unaops), un, len(operators.binops), bi, ctypes.byref(out)
                )
            )
            oid = int(out.value)
            self._opsets[key] = oid
        return oid

    def loss_code(self, options) -> int:
        """The `loss_kind` the C ABI takes for options' elementwise loss: the kind itself for the
        parameter-free losses (and HuberLoss(1)), else the code sr_register_loss returns."""
        kind, param = options.loss_kind, float(getattr(options, "loss_param", 0.0))
        if kind in (0, 1, 3, 9, 10, 11, 12, 14, 15, 16, 17) or (kind == 4 and param == 1.0):
            return kind
        key = (kind, param)
        codes = self.__dict__.setdefault("_loss_codes", {})
        if key not in codes:
            out = ctypes.c_int()
            _lib.check(_lib.lib.sr_register_loss(self.handle, kind, param, ctypes.byref(out)))
            codes[key] = int(out.value)
        return codes[key]

    def last_kernel_ms(self):
        a, b = ctypes.c_double(), ctypes.c_double()
        _lib.check(_lib.lib.sr_last_kernel_ms(self.handle, ctypes.byref(a), ctypes.byref(b)))
        return float(a.value), float(b.value)

    def last_phase_ms(self):
        """Host phases of the last eval_loss call: compile, upload+launch, wait, exact pass, finalize."""
        out = (ctypes.c_double * 6)()
        _lib.check(_lib.lib.sr_last_phase_ms(self.handle, out, 6))
        return [float(v) for v in out[:5]]

    def set_tuning(self, name, value):
        """Run-time tuning knob (include/sr_amd.h lists them): "derived", "probe", "stress_probe",
        "code_cache", "timing", "rows_per_lane", "balance", "fused_reduce", "exact_w", "exact_g", "fold_seg",
        "ref_fold" (the in-order loss fold: 1 default, 0 the f64 sums), "fold_seg_max" / "fold_rows_max"
        (the longest row block / fold folded: past them a call keeps the f64 sums — these three are the
        knobs results depend on), "fold_store_mb", "fold_slot_mb", "fold_delta_log2"; tests:
        "inject_failure*", "debug_hint_regrow", "fold_debug_fail"."""
        _lib.check(_lib.lib.sr_set_tuning(self.handle, name.encode(), int(value)))

    def last_derived_columns(self):
        """Derived columns (unary(feature) nodes evaluated once) used by the last eval_loss call."""
        n = ctypes.c_int(0)
        _lib.check(_lib.lib.sr_tuning_info(self.handle, ctypes.byref(n), None))
        return int(n.value)

    def last_exact_trees(self):
        """Trees of the last eval_loss call that went through the exact-sum pass (flagged BIG)."""
        n = ctypes.c_int64(0)
        _lib.check(_lib.lib.sr_tuning_info(self.handle, None, ctypes.byref(n)))
        return int(n.value)

    def last_ref_fold(self):
        """The last eval_loss call's in-order loss fold (csrc/sr_fold_dev.h): {path: 0 none / 1 stored
        losses / 2 FOLD-mode pass, folded: trees whose loss is the exact fold, fallback: trees folded
        through the prediction pass instead, kernel_ms: the fold launches' device time}."""
        p, a, b, ms = ctypes.c_int(0), ctypes.c_int64(0), ctypes.c_int64(0), ctypes.c_double(0.0)
        _lib.check(_lib.lib.sr_ref_fold_info(self.handle, ctypes.byref(p), ctypes.byref(a), ctypes.byref(b),
                                             ctypes.byref(ms)))
        return {"path": int(p.value), "folded": int(a.value), "fallback": int(b.value), "kernel_ms": float(ms.value)}

    def last_exact_kernel_ms(self):
        """Device time of the last eval_loss call's exact-sum pass (ms)."""
        out = (ctypes.c_double * 7)()
        _lib.check(_lib.lib.sr_last_phase_ms(self.handle, out, 7))
        return float(out[6])

    def last_rows_per_lane(self):
        """Rows per lane of the last call's interpreter kernel (8 or 16 for f32 BASIC loss)."""
        out = (ctypes.c_double * 8)()
        _lib.check(_lib.lib.sr_last_phase_ms(self.handle, out, 8))
        return int(out[7])

    def last_busy_ms(self):
        """Device-busy time of the last call's interpreter launches: the union of their intervals (ms)."""
        out = (ctypes.c_double * 9)()
        _lib.check(_lib.lib.sr_last_phase_ms(self.handle, out, 9))
        return float(out[8])

    def last_fold_trees(self):
        """Trees of the last eval_loss call whose loss fold was computed in row order (the reference's
        T-precision fold near overflow: csrc/sr_fold.h)."""
        out = (ctypes.c_double * 10)()
        _lib.check(_lib.lib.sr_last_phase_ms(self.handle, out, 10))
        return int(out[9])

    def last_fold_info(self):
        """The last eval_loss call's in-order loss folds: (trees folded, segments folded row by row,
        segment length in rows; 0 = one scan over every row) — sr_last_phase_ms out[9..11]."""
        out = (ctypes.c_double * 12)()
        _lib.check(_lib.lib.sr_last_phase_ms(self.handle, out, 12))
        return int(out[9]), int(out[10]), int(out[11])

    def last_fold_ms(self):
        """The last call's in-order loss fold, device ms (HIP events): {pred, segsum, segtab, chain}."""
        out = (ctypes.c_double * 16)()
        _lib.check(_lib.lib.sr_last_phase_ms(self.handle, out, 16))
        return dict(zip(("pred", "segsum", "segtab", "chain"), (float(v) for v in out[12:16])))

    def last_grad_info(self):
        """The last gradient call's tangent kernels per bucket (1, 2, 4, 8, 16 tangents): list of dicts
        {kt, kernel_ms, flops, items, rows_per_lane} (csrc: sr_last_grad_info)."""
        import numpy as np

        ms, fl = np.zeros(5), np.zeros(5)
        it = np.zeros(5, dtype=np.int64)
        rp = np.zeros(5, dtype=np.int32)
        p = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
        _lib.check(_lib.lib.sr_last_grad_info(self.handle, 5, p(ms), p(fl), p(it), p(rp)))
        return [dict(kt=k, kernel_ms=float(ms[b]), flops=float(fl[b]), items=int(it[b]), rows_per_lane=int(rp[b]))
                for b, k in enumerate((1, 2, 4, 8, 16))]

    def last_launches(self):
        """Interpreter launches of the last eval_loss call (chunked compile/launch pipeline)."""
        out = (ctypes.c_double * 6)()
        _lib.check(_lib.lib.sr_last_phase_ms(self.handle, out, 6))
        return int(out[5])

    def close(self):
        if self.handle:
            _lib.lib.sr_shutdown(self.handle)
            self.handle = None


def default_device() -> int:
    return int(os.environ.get("SR_AMD_DEVICE", os.environ.get("LOCAL_RANK", "0")))


def get_lane_context(lane: int, device: int | None = None) -> DeviceContext:
    """Scoring lane ``lane`` of a device: lane 0 is get_context(device); further lanes are contexts
    of their own (own streams and staging buffers), cached for the process."""
    if lane == 0:
        return get_context(device)
    dev = default_device() if device is None else int(device)
    with _lock:
        ctx = _lane_contexts.get((dev, lane))
        if ctx is None:
            ctx = DeviceContext(dev)
            _lane_contexts[(dev, lane)] = ctx
        return ctx


def get_context(device: int | None = None) -> DeviceContext:
    dev = default_device() if device is None else int(device)
    with _lock:
        ctx = _contexts.get(dev)
        if ctx is None:
            ctx = DeviceContext(dev)
            _contexts[dev] = ctx
        return ctx


def peek_context(device: int | None = None):
    """This process's context for `device` if one exists (no device call otherwise), else None."""
    dev = default_device() if device is None else int(device)
    with _lock:
        return _contexts.get(dev)


def device_available() -> bool:
    return _lib.device_count() > 0
