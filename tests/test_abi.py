"""CPU: the C-ABI library loads, exports every symbol include/sr_amd.h declares, and its host-only
entry points behave (no kernel launches here)."""
import ctypes
import os
import re

import numpy as np

from sr_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared_functions():
    with open(os.path.join(ROOT, "include", "sr_amd.h")) as f:
        src = f.read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(sr_[a-z0-9_]+)\s*\(", src)))


def test_header_symbols_exported():
    declared = _declared_functions()
    assert len(declared) >= 15
    lib = ctypes.CDLL(_lib.LIB_PATH)
    missing = [s for s in declared if not hasattr(lib, s)]
    assert not missing, missing
    assert set(declared) == set(_lib.EXPORTED_SYMBOLS)


def test_version_and_error_string():
    assert _lib.lib.sr_version() == 2
    rc = _lib.lib.sr_shutdown(None)
    assert rc == 0
    h = ctypes.c_void_p()
    rc = _lib.lib.sr_register_opset(None, 0, None, 0, None, ctypes.byref(ctypes.c_int()))
    assert rc == _lib.SR_ERR_INVALID_ARG
    assert "NULL" in _lib.last_error()
    del h


def test_init_without_gpu_fails_cleanly():
    if _lib.device_count() > 0:
        return  # on a GPU box this is covered by the gpu tests
    h = ctypes.c_void_p()
    rc = _lib.lib.sr_init(0, ctypes.byref(h))
    assert rc == _lib.SR_ERR_NO_DEVICE
    assert not h.value


def _finalize(dtype, sums, flags, denom, lst=None, list_ok=None):
    nt = len(sums)
    sums = np.ascontiguousarray(sums, dtype=np.float64)
    flags = np.ascontiguousarray(flags, dtype=np.uint32)
    out = np.empty(nt, dtype=np.float32 if dtype == _lib.SR_DTYPE_F32 else np.float64)
    comp = np.empty(nt, dtype=np.uint8)
    lst = None if lst is None else np.ascontiguousarray(lst, dtype=np.int64)
    ok = None if list_ok is None else np.ascontiguousarray(list_ok, dtype=np.uint8)
    p = lambda a: None if a is None else a.ctypes.data_as(ctypes.c_void_p)
    _lib.check(_lib.lib.sr_finalize_losses(dtype, nt, p(sums), p(flags), denom, p(lst),
                                           0 if lst is None else len(lst), p(ok), p(out), p(comp)))
    return out, comp.astype(bool)


def test_finalize_combines_partials():
    # tree0 fine, tree1 non-finite, tree2 static-bad, tree3 "big" but its Julia sums are finite,
    # tree4 big and one Julia sum overflows
    sums = [10.0, 5.0, 0.0, 8.0, 8.0]
    flags = [0, _lib.SR_FLAG_NONFINITE, _lib.SR_FLAG_STATIC | _lib.SR_FLAG_NONFINITE, _lib.SR_FLAG_BIG,
             _lib.SR_FLAG_BIG]
    loss, comp = _finalize(_lib.SR_DTYPE_F32, sums, flags, 4.0, lst=[3, 4], list_ok=[1, 0])
    assert list(comp) == [True, False, False, True, False]
    assert loss[0] == np.float32(2.5)
    assert np.isinf(loss[1]) and np.isinf(loss[2]) and np.isinf(loss[4])
    assert loss[3] == np.float32(2.0)


def test_finalize_rejects_bad_list():
    sums = np.zeros(2)
    flags = np.zeros(2, dtype=np.uint32)
    out = np.empty(2, dtype=np.float32)
    comp = np.empty(2, dtype=np.uint8)
    lst = np.array([5], dtype=np.int64)
    ok = np.ones(1, dtype=np.uint8)
    rc = _lib.lib.sr_finalize_losses(_lib.SR_DTYPE_F32, 2, sums.ctypes.data_as(ctypes.c_void_p),
                                     flags.ctypes.data_as(ctypes.c_void_p), 1.0, lst.ctypes.data_as(ctypes.c_void_p),
                                     1, ok.ctypes.data_as(ctypes.c_void_p), out.ctypes.data_as(ctypes.c_void_p),
                                     comp.ctypes.data_as(ctypes.c_void_p))
    assert rc == _lib.SR_ERR_INVALID_ARG
