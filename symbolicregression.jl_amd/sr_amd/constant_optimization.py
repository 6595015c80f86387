"""Batched constant optimisation (reference src/ConstantOptimization.jl), on the native optimiser.

The reference optimises one member at a time: ``optimize_constants`` (:29-59) runs
``Optim.optimize`` with ``BFGS(linesearch=BackTracking())`` (Newton for a single constant) from the
current constants and from ``optimizer_nrestarts`` perturbed starts ``x0 .* (1 + eps/2)``
(:77-116), keeps the best, and adopts it only if it beats the starting loss.  The library's
``sr_optimize_constants_batch`` (csrc/sr_constopt.h, csrc/sr_search.cpp) runs every tree of a
batch through the same algorithm in lock-step: each round of line-search trials is ONE batched
loss launch and each gradient ONE ``sr_eval_grad_batch`` launch for all trees still iterating, so a
whole population's constant optimisation costs a few dozen device launches.  The native search
engine uses the same optimiser for ``optimize_and_simplify_population``.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from .device import get_context


def device_optimizer_supported(options) -> bool:
    """The device path runs the reference's default optimiser only: Optim.BFGS with BackTracking
    (Newton for one constant, as optimize_constants chooses; src/ConstantOptimization.jl:38-56).  A
    caller with another ``optimizer_algorithm`` keeps the reference's CPU optimize_constants (the
    Julia glue's gate)."""
    return getattr(options, "optimizer_algorithm", "BFGS") == "BFGS"


def optimize_constants_batch(trees, dataset, options, rng=None, *, iterations=None, nrestarts=None, ctx=None,
                             f_calls_limit=None):
    """Optimise the constants of every tree of ``trees`` (TreeBatch or Nodes) on ``dataset``.

    Returns ``(new_batch, losses, improved, num_evals)``: the batch with adopted constants, the
    loss of each tree after optimisation (the starting loss when not improved), which trees improved
    (``result.minimum < baseline``), and the reference's ``num_evals`` accounting (objective calls x
    dataset fraction, +1 for the re-evaluation of an improved member, src/ConstantOptimization.jl:92-109).
    ``rng`` (numpy Generator) seeds the restart perturbations.  ``iterations`` / ``f_calls_limit``
    default to the options' ``optimizer_iterations`` / ``optimizer_f_calls_limit`` (Optim.Options,
    src/Options.jl:988-997); a non-BFGS ``optimizer_algorithm`` raises NotImplementedError (the
    reference's CPU optimiser is the caller's path for it).
    """
    from .loss import _as_batch

    if not device_optimizer_supported(options):
        raise NotImplementedError(f"optimizer_algorithm={options.optimizer_algorithm!r} runs on the reference's CPU "
                                  "optimize_constants; the device optimiser is BFGS + BackTracking")
    ctx = ctx or get_context()
    iterations = iterations if iterations is not None else getattr(options, "optimizer_iterations", 8)
    f_calls_limit = f_calls_limit if f_calls_limit is not None else getattr(options, "optimizer_f_calls_limit", 10_000)
    nrestarts = nrestarts if nrestarts is not None else getattr(options, "optimizer_nrestarts", 2)
    full = dataset.full
    tb = _as_batch(trees, full.dtype)
    nt = tb.n_trees
    seed = int((rng if rng is not None else np.random.default_rng()).integers(0, 2 ** 63))
    consts = np.zeros(max(1, int(np.count_nonzero(tb.constant_mask()))), dtype=full.dtype)
    losses = np.zeros(max(1, nt), dtype=full.dtype)
    improved = np.zeros(max(1, nt), dtype=np.uint8)
    f_calls = np.zeros(max(1, nt), dtype=np.int64)
    idx = dataset.indices
    rows = None if idx is None else np.ascontiguousarray(idx, dtype=np.int64)
    p = lambda a: None if a is None else a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    s = tb.to_struct()
    _lib.check(_lib.lib.sr_optimize_constants_batch(
        ctx.handle, full.device_handle(ctx), ctx.opset_id(options.operators), ctypes.byref(s), p(rows),
        0 if rows is None else rows.size, ctx.loss_code(options), int(iterations), int(f_calls_limit), int(nrestarts),
        ctypes.c_uint64(seed), p(consts), p(losses), p(improved), p(f_calls)))
    n_const = int(np.count_nonzero(tb.constant_mask()))
    new_tb = tb.with_constants(consts[:n_const])
    imp = improved[:nt].astype(bool)
    num_evals = (f_calls[:nt] + imp.astype(np.int64)) * dataset.dataset_fraction()
    return new_tb, losses[:nt].copy(), imp, num_evals


def optimize_constants_callbacks(trees, loss_fn, grad_fn, *, dtype=np.float64, seed=0, iterations=8, nrestarts=2,
                                 rows=None, f_calls_limit=0):
    """The same batched optimiser with CPU scorers (``sr_optimize_constants_callbacks``; test seam):
    loss_fn(TreeBatch, rows) -> losses, grad_fn(TreeBatch, rows) -> (losses, gradients).  The restart
    draws come from ``seed`` exactly as ``optimize_constants_batch``'s.  Returns (new_batch, losses,
    improved, f_calls)."""
    from .loss import _as_batch
    from .search import make_callbacks

    tb = _as_batch(trees, dtype)
    nt = tb.n_trees
    n_const = int(np.count_nonzero(tb.constant_mask()))
    consts = np.zeros(max(1, n_const), dtype=dtype)
    losses = np.zeros(max(1, nt), dtype=dtype)
    improved = np.zeros(max(1, nt), dtype=np.uint8)
    f_calls = np.zeros(max(1, nt), dtype=np.int64)
    cbs = make_callbacks(dtype, loss_fn, grad_fn)
    r = None if rows is None else np.ascontiguousarray(rows, dtype=np.int64)
    p = lambda a: None if a is None else a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    s = tb.to_struct()
    _lib.check(_lib.lib.sr_optimize_constants_callbacks(
        _lib.SR_DTYPE_F32 if np.dtype(dtype) == np.float32 else _lib.SR_DTYPE_F64, ctypes.byref(s), p(r),
        0 if r is None else r.size, int(iterations), int(f_calls_limit), int(nrestarts), ctypes.c_uint64(int(seed)),
        cbs[0], cbs[1], None,
        p(consts), p(losses), p(improved), p(f_calls)))
    return tb.with_constants(consts[:n_const]), losses[:nt].copy(), improved[:nt].astype(bool), f_calls[:nt].copy()
