"""Row-sharded scoring across GPUs (one process per GPU, torch.distributed over RCCL).

Each rank holds one row shard of the dataset (HBM-resident), scores every tree on it
(`sr_eval_loss_partials`: per-tree f64 Σ loss and flag bits), and the ranks combine the partials
with all-reduces — SUM for the sums, MAX per flag bit — before `sr_finalize_losses` turns them into
losses.  Trees that came close to overflowing a checked array sum (BIG only) need the exact per-check
sums of every shard: one more all-reduce of `sr_exact_check_partials`.  This is the path's only
exchange step; at 10k trees it moves 8 B + 12 B per tree.

`partials_fn` / `exact_fn` default to the GPU calls; tests inject CPU stand-ins to exercise the
combine logic with the gloo backend.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from .device import get_context
from .loss import _as_batch

FLAG_BITS = (_lib.SR_FLAG_NONFINITE, _lib.SR_FLAG_BIG, _lib.SR_FLAG_STATIC)


def gpu_partials(tb, shard, options, n_total, ctx=None):
    """This rank's per-tree (Σ loss f64, flags u32) on its row shard (GPU)."""
    ctx = ctx or get_context()
    nt = tb.n_trees
    sums = np.zeros(nt, dtype=np.float64)
    flags = np.zeros(nt, dtype=np.uint32)
    s = tb.to_struct()
    _lib.check(_lib.lib.sr_eval_loss_partials(
        ctx.handle, shard.device_handle(ctx), ctx.opset_id(options.operators), ctypes.byref(s), int(n_total),
        ctx.loss_code(options), sums.ctypes.data_as(ctypes.c_void_p), flags.ctypes.data_as(ctypes.c_void_p), 0))
    return sums, flags


def gpu_exact(tb, shard, options, tree_list, ctx=None):
    """This rank's exact per-check array sums for the listed trees (GPU): [n_list, max_checks]."""
    ctx = ctx or get_context()
    oid = ctx.opset_id(options.operators)
    s = tb.to_struct()
    m = ctypes.c_int()
    _lib.check(_lib.lib.sr_max_checks(ctx.handle, oid, ctypes.byref(s), ctypes.byref(m)))
    mc = int(m.value)
    lst = np.ascontiguousarray(tree_list, dtype=np.int64)
    out = np.zeros((lst.size, mc), dtype=np.float64)
    if lst.size and mc:
        _lib.check(_lib.lib.sr_exact_check_partials(
            ctx.handle, shard.device_handle(ctx), oid, ctypes.byref(s), lst.ctypes.data_as(ctypes.c_void_p),
            lst.size, mc, out.ctypes.data_as(ctypes.c_void_p)))
    return out


def finalize(dtype, sums, flags, denom, tree_list=None, check_sums=None):
    """Host combine (C ABI `sr_finalize_losses`): losses[T], complete[bool]."""
    nt = len(sums)
    sums = np.ascontiguousarray(sums, dtype=np.float64)
    flags = np.ascontiguousarray(flags, dtype=np.uint32)
    out = np.empty(nt, dtype=dtype)
    comp = np.empty(nt, dtype=np.uint8)
    p = lambda a: None if a is None else a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    lst = None if tree_list is None or len(tree_list) == 0 else np.ascontiguousarray(tree_list, dtype=np.int64)
    cs = None if lst is None else np.ascontiguousarray(check_sums, dtype=np.float64)
    mc = 0 if cs is None else int(cs.shape[1])
    _lib.check(_lib.lib.sr_finalize_losses(
        _lib.SR_DTYPE_F32 if np.dtype(dtype) == np.float32 else _lib.SR_DTYPE_F64, nt, p(sums), p(flags),
        float(denom), p(lst), 0 if lst is None else lst.size, mc, p(cs), p(out), p(comp)))
    return out, comp.astype(bool)


def _all_reduce_np(dist, arr, op, group):
    import torch

    t = torch.from_numpy(np.ascontiguousarray(arr))
    dev = _reduce_device(dist, group)
    if dev is not None:
        t = t.to(dev)
    dist.all_reduce(t, op=op, group=group)
    return t.cpu().numpy()


def _reduce_device(dist, group):
    # RCCL ("nccl") reduces device tensors; gloo reduces host tensors
    if dist.get_backend(group) == "nccl":
        import torch

        return torch.device("cuda", torch.cuda.current_device())
    return None


def eval_loss_sharded(trees, shard, options, n_total, *, denom=None, group=None, partials_fn=None, exact_fn=None):
    """Losses of every tree over the union of all ranks' row shards -> (losses[T], complete[bool]).

    `denom`: global denominator (Σ rows, or Σ weights); defaults to `n_total` for unweighted data.
    """
    import torch.distributed as dist

    full = shard.full
    tb = _as_batch(trees, full.dtype)
    partials_fn = partials_fn or (lambda tb_: gpu_partials(tb_, shard, options, n_total))
    exact_fn = exact_fn or (lambda tb_, lst: gpu_exact(tb_, shard, options, lst))
    sums, flags = partials_fn(tb)
    sums = _all_reduce_np(dist, sums, dist.ReduceOp.SUM, group)
    bits = np.stack([(flags & b) != 0 for b in FLAG_BITS]).astype(np.int32)
    bits = _all_reduce_np(dist, bits, dist.ReduceOp.MAX, group)
    flags = np.zeros(tb.n_trees, dtype=np.uint32)
    for k, b in enumerate(FLAG_BITS):
        flags |= np.where(bits[k] != 0, np.uint32(b), np.uint32(0))
    big = np.nonzero(((flags & (_lib.SR_FLAG_NONFINITE | _lib.SR_FLAG_STATIC)) == 0) & ((flags & _lib.SR_FLAG_BIG) != 0))[0]
    cs = None
    if big.size:
        cs = _all_reduce_np(dist, exact_fn(tb, big), dist.ReduceOp.SUM, group)
    if denom is None:
        if full.weights is not None:
            local = np.array([float(np.sum(full.weights, dtype=np.float64))])
            denom = float(_all_reduce_np(dist, local, dist.ReduceOp.SUM, group)[0])
        else:
            denom = float(n_total)
    return finalize(full.dtype, sums, flags, denom, big, cs)
