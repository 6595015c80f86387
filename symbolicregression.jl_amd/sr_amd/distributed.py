"""Multi-GPU scoring: rows sharded (C4) and trees sharded, one process per GPU.

The data path's exchanges run inside the library on its own RCCL communicator over xGMI
(`init_device_comm` → C ABI `sr_comm_*`); torch.distributed is used only as a CPU channel (a gloo
group: the 128-byte RCCL unique id, barriers, small host objects).  torch never touches the GPU:
its bundled HIP runtime cannot share the device with the library's in one process.

Row sharding, `eval_loss_sharded`: rank r holds global rows [Σ_{q<r} n_q, Σ_{q<=r} n_q).  With a
device communicator the whole step is ONE library call (`sr_eval_loss_sharded`): the shard runs
the single-GPU launch pipeline, its packed [5, n_trees] partials (Σ loss, then the NONFINITE / BIG /
STATIC / ELEMINF flag bits as 0/1) are summed by one in-place RCCL all-reduce, losses are finalized on
the device, the rare BIG trees get DynamicExpressions' exact isfinite(sum(x)) verdict in Julia's
pairwise order over the GLOBAL rows (each rank folds the leaf blocks it holds; the folds are
all-gathered; `sr_jsum_finite`'s recursion-order combine), and the rarer trees whose T-precision loss
fold may overflow are folded in row order across the shards.

`init_host_comm` gives the library the same collectives over the gloo group instead of RCCL
(`sr_comm_init_host`): the library's own sharded code then runs with several ranks on one GPU (the
multi-rank tests on a one-GPU box).

Tree sharding, `eval_loss_tree_sharded`: the dataset is replicated, the trees are dealt over the
ranks by size, each rank scores its share, one all-reduce hands every rank every result
(`sr_eval_loss_tree_sharded`).

Without a device communicator (tests on CPU: `partials_fn` / `exact_fn` / `score_fn` stand-ins for
the GPU calls) the same protocols run over the gloo group on host arrays.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from .device import get_context, peek_context
from .loss import _as_batch


def _dtype_code(dtype):
    return _lib.SR_DTYPE_F32 if np.dtype(dtype) == np.float32 else _lib.SR_DTYPE_F64


def _require_gloo(group):
    import torch.distributed as dist

    backend = dist.get_backend(group)
    if backend != "gloo":
        # an "nccl" group would make torch initialise its own HIP runtime on the GPU, which cannot share
        # the device with the library's; the data path's collectives are the library's own RCCL
        raise RuntimeError(f"sr_amd.distributed needs a gloo process group as its CPU channel (got {backend!r}); "
                           "the device collectives run on the library's RCCL communicator (init_device_comm)")


N_PACKED = 5  # rows of the packed partials: Σ loss, NONFINITE, BIG, STATIC, ELEMINF


def gpu_partials_packed(tb, shard, options, n_total, ctx=None):
    """This rank's packed partials [5, n_trees] f64 on its row shard (GPU), on the host."""
    ctx = ctx or get_context()
    nt = tb.n_trees
    s = tb.to_struct()
    out = np.zeros((N_PACKED, nt), dtype=np.float64)
    _lib.check(_lib.lib.sr_eval_loss_partials_packed(
        ctx.handle, shard.device_handle(ctx), ctx.opset_id(options.operators), ctypes.byref(s), int(n_total),
        ctx.loss_code(options), out.ctypes.data_as(ctypes.c_void_p), 0))
    return out


SR_COMM_ID_BYTES = 128


def init_device_comm(group=None, ctx=None):
    """Create this rank's RCCL communicator inside the library (C ABI sr_comm_*) over the ranks of
    `group` (a gloo group: it only broadcasts rank 0's unique id).  The communicator's size and rank
    must equal the group's; after this the sharded calls exchange on the devices over xGMI."""
    import torch.distributed as dist

    _require_gloo(group)
    ctx = ctx or get_context()
    buf = ctypes.create_string_buffer(SR_COMM_ID_BYTES)
    if dist.get_rank(group) == 0:
        _lib.check(_lib.lib.sr_comm_unique_id(ctypes.cast(buf, ctypes.c_void_p)))
    obj = [bytes(buf.raw)]
    dist.broadcast_object_list(obj, src=0, group=group)
    raw = ctypes.create_string_buffer(obj[0], SR_COMM_ID_BYTES)
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    _lib.check(_lib.lib.sr_comm_init(ctx.handle, world, rank, ctypes.cast(raw, ctypes.c_void_p)))
    info = comm_info(ctx)
    if (info["nranks"], info["rank"]) != (world, rank):
        raise RuntimeError(f"RCCL communicator is rank {info['rank']} of {info['nranks']}, group says {rank} of {world}")
    ctx.has_comm = True
    ctx.comm_world, ctx.comm_rank = world, rank
    return ctx


def init_host_comm(group=None, ctx=None):
    """The library's sharded calls over the gloo `group` instead of RCCL (C ABI sr_comm_init_host): the
    library stages each collective's buffer through host memory and calls back into torch.distributed
    (all_reduce of float64 / all_gather of bytes).  The same C++ code path as with RCCL, so several
    ranks can share one GPU (tests)."""
    import torch
    import torch.distributed as dist

    _require_gloo(group)
    ctx = ctx or get_context()
    world, rank = dist.get_world_size(group), dist.get_rank(group)

    def allreduce(_user, buf, n):
        try:
            a = np.ctypeslib.as_array(buf, shape=(int(n),))
            t = torch.from_numpy(a.copy())
            dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
            a[:] = t.numpy()
            return 0
        except Exception:  # noqa: BLE001 - reported to the library as a failed collective
            return 1

    def allgather(_user, send, recv, nbytes):
        try:
            nb = int(nbytes)
            src = np.frombuffer((ctypes.c_char * nb).from_address(send), dtype=np.uint8).copy()
            parts = [torch.empty(nb, dtype=torch.uint8) for _ in range(world)]
            dist.all_gather(parts, torch.from_numpy(src), group=group)
            dst = np.frombuffer((ctypes.c_char * (nb * world)).from_address(recv), dtype=np.uint8)
            for r, part in enumerate(parts):
                dst[r * nb:(r + 1) * nb] = part.numpy()
            return 0
        except Exception:  # noqa: BLE001
            return 1

    ctx._host_comm_cbs = (_lib.HOST_ALLREDUCE_FN(allreduce), _lib.HOST_ALLGATHER_FN(allgather))
    _lib.check(_lib.lib.sr_comm_init_host(ctx.handle, world, rank, ctx._host_comm_cbs[0], ctx._host_comm_cbs[1], None))
    info = comm_info(ctx)
    if (info["nranks"], info["rank"], info.get("transport")) != (world, rank, "host"):
        raise RuntimeError(f"host communicator is rank {info['rank']} of {info['nranks']}, group says {rank} of {world}")
    ctx.has_comm = True
    ctx.comm_world, ctx.comm_rank = world, rank
    return ctx


def destroy_device_comm(ctx=None):
    ctx = ctx or get_context()
    _lib.check(_lib.lib.sr_comm_destroy(ctx.handle))
    ctx.has_comm = False


def comm_info(ctx=None):
    """{"nranks", "rank"} as RCCL reports them, and the files of the HIP runtime / RCCL in use."""
    ctx = ctx or get_context()
    n, r = ctypes.c_int(), ctypes.c_int()
    buf = ctypes.create_string_buffer(4096)
    _lib.check(_lib.lib.sr_comm_info(ctx.handle, ctypes.byref(n), ctypes.byref(r), buf, len(buf)))
    out = dict(kv.split("=", 1) for kv in buf.value.decode().split(";") if "=" in kv)
    out.update(nranks=int(n.value), rank=int(r.value))
    return out


def _check_group(ctx, group):
    """The device communicator must span exactly the ranks of `group` (else the sums and the host-side
    verdicts would come from different sets of ranks)."""
    import torch.distributed as dist

    if (getattr(ctx, "comm_world", None), getattr(ctx, "comm_rank", None)) != (dist.get_world_size(group),
                                                                              dist.get_rank(group)):
        raise RuntimeError("the device communicator was created over another group of ranks")


def gpu_partials_allreduce(tb, shard, options, n_total, ctx=None):
    """Every rank's packed partials [5, n_trees], summed on the devices by the library's
    communicator (`sr_eval_loss_partials_allreduce`) -> numpy on every rank."""
    ctx = ctx or get_context()
    nt = tb.n_trees
    s = tb.to_struct()
    out = np.zeros((N_PACKED, max(nt, 1)), dtype=np.float64)
    _lib.check(_lib.lib.sr_eval_loss_partials_allreduce(
        ctx.handle, shard.device_handle(ctx), ctx.opset_id(options.operators), ctypes.byref(s), int(n_total),
        ctx.loss_code(options), out.ctypes.data_as(ctypes.c_void_p)))
    return out[:, :nt]


def jsum_ranges(row_offset, n_local, n_total):
    """(lo, hi, leaf, head) of the row ranges a shard folds for the exact check (C ABI)."""
    n = ctypes.c_int64()
    _lib.check(_lib.lib.sr_jsum_range_count(int(row_offset), int(n_local), int(n_total), ctypes.byref(n)))
    lo, hi, leaf = (np.zeros(n.value, dtype=np.int64) for _ in range(3))
    head = np.zeros(n.value, dtype=np.uint8)
    p = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    _lib.check(_lib.lib.sr_jsum_ranges(int(row_offset), int(n_local), int(n_total), p(lo), p(hi), p(leaf), p(head)))
    return lo, hi, leaf, head.astype(bool)


def gpu_jsum(tb, shard, options, tree_list, max_checks, row_offset, n_total, ctx=None):
    """This rank's Julia-order folds of every checked array of the listed trees over its ranges:
    [n_list, max_checks, n_ranges] (dataset dtype)."""
    ctx = ctx or get_context()
    oid = ctx.opset_id(options.operators)
    s = tb.to_struct()
    lst = np.ascontiguousarray(tree_list, dtype=np.int64)
    n_ranges = len(jsum_ranges(row_offset, shard.n, n_total)[0])
    out = np.zeros((lst.size, max_checks, n_ranges), dtype=shard.full.dtype)
    if lst.size and max_checks:
        _lib.check(_lib.lib.sr_jsum_partials(
            ctx.handle, shard.device_handle(ctx), oid, ctypes.byref(s), lst.ctypes.data_as(ctypes.c_void_p),
            lst.size, max_checks, int(row_offset), int(n_total), out.ctypes.data_as(ctypes.c_void_p)))
    return out


def gpu_max_checks(tb, options, ctx=None):
    ctx = ctx or get_context()
    s = tb.to_struct()
    m = ctypes.c_int()
    _lib.check(_lib.lib.sr_max_checks(ctx.handle, _dtype_code(tb.val.dtype), ctx.opset_id(options.operators),
                                      ctypes.byref(s), ctypes.byref(m)))
    return int(m.value)


def jsum_finite(dtype, n_total, row_offsets, rank_vals):
    """isfinite(Julia sum) per array from every shard's folds (C ABI sr_jsum_finite).
    rank_vals[r]: [n_arrays, n_ranges_r] of shard r = [row_offsets[r], row_offsets[r + 1])."""
    offs = np.ascontiguousarray(row_offsets, dtype=np.int64)
    vals = [np.ascontiguousarray(v, dtype=dtype) for v in rank_vals]
    n_arrays = int(vals[0].shape[0]) if vals else 0
    ptrs = (ctypes.c_void_p * len(vals))(*[v.ctypes.data_as(ctypes.c_void_p) for v in vals])
    out = np.zeros(n_arrays, dtype=np.uint8)
    _lib.check(_lib.lib.sr_jsum_finite(_dtype_code(dtype), int(n_total), len(vals), offs.ctypes.data_as(ctypes.c_void_p),
                                       ptrs, n_arrays, out.ctypes.data_as(ctypes.c_void_p)))
    return out.astype(bool)


def finalize(dtype, sums, flags, denom, tree_list=None, list_ok=None):
    """Host combine (C ABI `sr_finalize_losses`): losses[T], complete[bool]."""
    nt = len(sums)
    sums = np.ascontiguousarray(sums, dtype=np.float64)
    flags = np.ascontiguousarray(flags, dtype=np.uint32)
    out = np.empty(nt, dtype=dtype)
    comp = np.empty(nt, dtype=np.uint8)
    p = lambda a: None if a is None else a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    lst = None if tree_list is None or len(tree_list) == 0 else np.ascontiguousarray(tree_list, dtype=np.int64)
    ok = None if lst is None else np.ascontiguousarray(list_ok, dtype=np.uint8)
    _lib.check(_lib.lib.sr_finalize_losses(_dtype_code(dtype), nt, p(sums), p(flags), float(denom), p(lst),
                                           0 if lst is None else lst.size, p(ok), p(out), p(comp)))
    return out, comp.astype(bool)


def unpack_flags(packed):
    """[5, n] summed partials -> (Σ loss f64, flag words u32): a bit is set if any rank set it."""
    packed = np.asarray(packed, dtype=np.float64)
    flags = np.zeros(packed.shape[1], dtype=np.uint32)
    for row, bit in ((1, _lib.SR_FLAG_NONFINITE), (2, _lib.SR_FLAG_BIG), (3, _lib.SR_FLAG_STATIC),
                     (4, _lib.SR_FLAG_ELEMINF)):
        flags |= np.where(packed[row] > 0, np.uint32(bit), np.uint32(0))
    return packed[0].copy(), flags


def _allreduce_host(arr, group, op="sum"):
    import torch
    import torch.distributed as dist

    t = torch.from_numpy(np.ascontiguousarray(arr))
    dist.all_reduce(t, op=dist.ReduceOp.SUM if op == "sum" else dist.ReduceOp.MAX, group=group)
    return t.numpy()


def eval_loss_sharded(trees, shard, options, n_total=None, *, denom=None, group=None, partials_fn=None,
                      exact_fn=None):
    """Losses of every tree over the union of all ranks' row shards -> (losses[T], complete[bool]),
    the same on every rank.  Collective: every rank calls it with the same trees.

    With a library communicator (init_device_comm: RCCL; init_host_comm: gloo) this is one
    `sr_eval_loss_sharded` call.  Otherwise (CPU tests of the protocol, stand-ins for the GPU calls)
    the protocol runs here over the gloo `group` on host arrays: `partials_fn(tb)` -> this shard's
    packed [5, n_trees] partials (default: the GPU call), `exact_fn(tb, tree_list, max_checks,
    row_offset)` -> [n_list, max_checks, n_ranges] folds (default: the GPU call).  This host
    restatement finalizes through `sr_finalize_losses`, which applies only the elementwise +Inf flag
    (SR_FLAG_ELEMINF): NOT the overflow rule's bounds and NOT the in-order fold of the reference's
    T-precision loss sum, so a tree whose Float32 fold overflows while its f64 sum stays finite scores
    finite here but +Inf through the library's own sharded call (use a library
    communicator for the reference's L(Inf) verdicts).  A failure on one rank is
    all-reduced as an error word, so every rank raises instead of waiting in a collective.  `denom`
    applies to this restatement only (the library divides by the shards' n or Σw)."""
    import torch.distributed as dist

    full = shard.full
    tb = _as_batch(trees, full.dtype)
    ctx = peek_context()
    if partials_fn is None and exact_fn is None and getattr(ctx, "has_comm", False):
        if denom is not None:
            raise ValueError("the library's sharded call divides by the shards' own n or Σw; `denom` is not supported")
        _check_group(ctx, group)
        nt = tb.n_trees
        s = tb.to_struct()
        loss = np.empty(nt, dtype=full.dtype)
        comp = np.empty(nt, dtype=np.uint8)
        _lib.check(_lib.lib.sr_eval_loss_sharded(
            ctx.handle, shard.device_handle(ctx), ctx.opset_id(options.operators), ctypes.byref(s),
            ctx.loss_code(options), loss.ctypes.data_as(ctypes.c_void_p), comp.ctypes.data_as(ctypes.c_void_p)))
        if n_total is not None:
            sizes = [None] * dist.get_world_size(group)
            dist.all_gather_object(sizes, int(shard.n), group=group)
            if sum(sizes) != int(n_total):
                raise ValueError(f"n_total {n_total} != the shards' {sum(sizes)} rows")
        return loss, comp.astype(bool)

    _require_gloo(group)
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    sizes = [None] * world
    dist.all_gather_object(sizes, int(shard.n), group=group)
    offs = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
    if n_total is None:
        n_total = int(offs[-1])
    elif int(offs[-1]) != int(n_total):
        raise ValueError(f"n_total {n_total} != the shards' {int(offs[-1])} rows")
    partials_fn = partials_fn or (lambda tb_: gpu_partials_packed(tb_, shard, options, n_total))
    nt = tb.n_trees
    buf = np.zeros(N_PACKED * nt + 1, dtype=np.float64)
    err = None
    try:
        buf[:N_PACKED * nt] = np.asarray(partials_fn(tb), dtype=np.float64).reshape(-1)
    except Exception as e:  # noqa: BLE001 - every rank must still enter the collective
        err = e
        buf[:] = 0.0
        buf[-1] = 1.0
    # the path's one exchange step: every rank's [5, n_trees] partials (and error words), summed
    buf = _allreduce_host(buf, group)
    if err is not None:
        raise err
    if buf[-1] != 0.0:
        raise RuntimeError("the row-sharded step failed on a peer rank")
    sums, flags = unpack_flags(buf[:N_PACKED * nt].reshape(N_PACKED, nt))
    big = np.nonzero(((flags & (_lib.SR_FLAG_NONFINITE | _lib.SR_FLAG_STATIC)) == 0) &
                     ((flags & _lib.SR_FLAG_BIG) != 0))[0]
    ok = None
    if big.size:
        # rare: exact Julia-order verdict over the global rows
        try:
            if exact_fn is None:
                # only the BIG trees are compiled again (a sub-batch: the check numbering is per tree)
                sub = tb.take(big)
                mc = gpu_max_checks(sub, options)
                mine = np.ascontiguousarray(gpu_jsum(sub, shard, options, np.arange(big.size), mc, int(offs[rank]),
                                                     n_total))
            else:
                mine = np.ascontiguousarray(exact_fn(tb, big, 1, int(offs[rank])))
            payload = (None, mine)
        except Exception as e:  # noqa: BLE001
            payload = (repr(e), None)
        every = [None] * world
        dist.all_gather_object(every, payload, group=group)
        bad = [r for r, (e, _) in enumerate(every) if e is not None]
        if bad:
            raise RuntimeError(f"the exact-sum pass failed on rank(s) {bad}: {every[bad[0]][0]}")
        mc = every[0][1].shape[1]
        fin = jsum_finite(full.dtype, n_total, offs, [v.reshape(big.size * mc, -1) for _, v in every])
        ok = fin.reshape(big.size, mc).all(axis=1).astype(np.uint8)
    if denom is None:
        if full.weights is not None:
            denom = float(_allreduce_host(np.array([np.sum(full.weights, dtype=np.float64)]), group)[0])
        else:
            denom = float(n_total)
    return finalize(full.dtype, sums, flags, denom, big, ok)


def tree_owners(tb, world):
    """Owner rank of every tree for tree sharding (the library's rule, sr_eval_loss_tree_sharded):
    trees sorted by node count (largest first, stable), dealt in snake order 0..N-1, N-1..0, ..."""
    sizes = np.diff(np.asarray(tb.offsets, dtype=np.int64))
    order = np.argsort(-sizes, kind="stable")
    k = np.arange(len(order))
    rnd, pos = k // world, k % world
    owner = np.where(rnd % 2 == 1, world - 1 - pos, pos)
    out = np.empty(len(order), dtype=np.int64)
    out[order] = owner
    return out


def eval_loss_tree_sharded(trees, dataset, options, *, group=None, score_fn=None):
    """Tree-sharded batched eval_loss: every rank holds the whole dataset; each scores
    the trees `tree_owners` gives it and every rank gets every (loss, complete).  Collective.
    With a device communicator: one `sr_eval_loss_tree_sharded` call (RCCL all-reduce of the results);
    otherwise over the gloo group with `score_fn(sub_batch) -> (losses, complete)` (default: the
    single-GPU `eval_loss_batch`)."""
    import torch.distributed as dist

    full = getattr(dataset, "full", dataset)
    tb = _as_batch(trees, full.dtype)
    ctx = peek_context()
    if score_fn is None and getattr(ctx, "has_comm", False):
        _check_group(ctx, group)
        nt = tb.n_trees
        s = tb.to_struct()
        loss = np.empty(nt, dtype=full.dtype)
        comp = np.empty(nt, dtype=np.uint8)
        _lib.check(_lib.lib.sr_eval_loss_tree_sharded(
            ctx.handle, dataset.device_handle(ctx), ctx.opset_id(options.operators), ctypes.byref(s),
            ctx.loss_code(options), loss.ctypes.data_as(ctypes.c_void_p), comp.ctypes.data_as(ctypes.c_void_p)))
        return loss, comp.astype(bool)

    _require_gloo(group)
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    if score_fn is None:
        from .loss import eval_loss_batch

        def score_fn(sub):
            return eval_loss_batch(sub, dataset, options)
    mine = np.nonzero(tree_owners(tb, world) == rank)[0]
    nt = tb.n_trees
    buf = np.zeros(2 * nt + 1, dtype=np.float64)
    err = None
    try:
        l, c = score_fn(tb.take(mine))
        buf[mine] = np.asarray(l, dtype=np.float64)
        buf[nt + mine] = np.asarray(c, dtype=np.float64)
    except Exception as e:  # noqa: BLE001 - every rank must still enter the collective
        err = e
        buf[:] = 0.0
        buf[-1] = 1.0
    buf = _allreduce_host(buf, group)
    if err is not None:
        raise err
    if buf[-1] != 0.0:
        raise RuntimeError("tree-sharded scoring failed on a peer rank")
    return buf[:nt].astype(full.dtype), buf[nt:2 * nt] != 0.0
