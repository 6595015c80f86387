"""GPU: the asynchronous loss call (sr_eval_loss_submit / sr_eval_loss_wait) and a second context on a
context's stream (sr_init_shared) — what the search's pipelined lanes run (csrc/sr_search.cpp
iterate_islands).  Two calls in flight on one stream give the synchronous call's bits; a second submit
on a busy context, and any other call on it, are refused until its wait."""
import ctypes

import numpy as np
import pytest

import sr_amd
from sr_amd import Dataset, Options, _lib, eval_loss_batch, flatten_trees, gen_random_population

pytestmark = pytest.mark.gpu


def _submit(ctx_handle, ds_handle, oid, tb, code, rows=None):
    s = tb.to_struct()
    loss = np.empty(tb.n_trees, dtype=np.float32)
    comp = np.empty(tb.n_trees, dtype=np.uint8)
    r = None if rows is None else np.ascontiguousarray(rows, dtype=np.int64)
    p = lambda a: None if a is None else a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    rc = _lib.lib.sr_eval_loss_submit(ctx_handle, ds_handle, oid, ctypes.byref(s), None, 1, p(r),
                                      0 if r is None else r.size, code, p(loss), p(comp))
    return rc, (s, r, loss, comp)  # (keep every array alive until the wait)


def test_two_calls_in_flight_on_one_stream_equal_the_synchronous_calls():
    opts = Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp", "log"])
    rng = np.random.default_rng(41)
    X = rng.uniform(0.5, 2.0, (5, 100_000)).astype(np.float32)
    y = (X[0] * X[1] * X[2] / (X[3] * X[4] ** 2 + 1)).astype(np.float32)
    ds = Dataset(X, y)
    tb1 = flatten_trees(gen_random_population(40, opts, 5, max_size=20, seed=41), np.float32)
    tb2 = flatten_trees(gen_random_population(300, opts, 5, max_size=25, seed=42), np.float32)
    rows = rng.integers(0, X.shape[1], 5000)
    ref1 = eval_loss_batch(tb1, ds, opts)
    ctx = sr_amd.get_context()
    h2 = ctypes.c_void_p()
    _lib.check(_lib.lib.sr_init_shared(ctx.handle, ctypes.byref(h2)))
    try:
        dsh = ds.device_handle(ctx)
        oid, code = ctx.opset_id(opts.operators), ctx.loss_code(opts)
        # the synchronous references, on the parent context (full data, and a row view)
        s2 = tb2.to_struct()
        l2 = np.empty(tb2.n_trees, dtype=np.float32)
        c2 = np.empty(tb2.n_trees, dtype=np.uint8)
        r64 = np.ascontiguousarray(rows, dtype=np.int64)
        _lib.check(_lib.lib.sr_eval_loss_batch(ctx.handle, dsh, oid, ctypes.byref(s2), r64.ctypes.data_as(ctypes.c_void_p),
                                               r64.size, code, l2.ctypes.data_as(ctypes.c_void_p),
                                               c2.ctypes.data_as(ctypes.c_void_p)))
        for rep in range(3):
            rc, a = _submit(ctx.handle, dsh, oid, tb1, code)
            _lib.check(rc)
            rc, b = _submit(h2, dsh, oid, tb2, code, rows)  # the shared context: the parent's dataset and opset
            _lib.check(rc)
            # a busy context refuses another submit and every other call until its wait
            rc_busy, _ = _submit(ctx.handle, dsh, oid, tb1, code)
            assert rc_busy != 0 and "pending" in _lib.lib.sr_last_error().decode()
            with pytest.raises(Exception):
                eval_loss_batch(tb1, ds, opts)
            order = (h2, ctx.handle) if rep % 2 else (ctx.handle, h2)  # either wait order
            for h in order:
                _lib.check(_lib.lib.sr_eval_loss_wait(h))
            assert np.array_equal(a[3].astype(bool), ref1[1]) and np.array_equal(a[2].view(np.uint32), ref1[0].view(np.uint32))
            assert np.array_equal(b[3], c2) and np.array_equal(b[2].view(np.uint32), l2.view(np.uint32))
        assert _lib.lib.sr_eval_loss_wait(ctx.handle) != 0  # nothing pending
        assert 0.1 < ref1[1].mean() < 0.95
    finally:
        _lib.lib.sr_shutdown(h2)
