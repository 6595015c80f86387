"""Scoring API mirrored from reference src/LossFunctions.jl, backed by the MI355X batch evaluator.

Single-tree functions keep the reference signatures (``eval_loss``, ``eval_cost``, ``loss_to_cost``,
``update_baseline_loss!`` -> ``update_baseline_loss_``); the batched entry points
(``eval_loss_batch`` / ``eval_cost_batch``) score a whole population in one device call — the
drop-in the reference's ``Population``/``finalize_costs``/reload call sites switch to.
"""
from __future__ import annotations

import ctypes
from typing import Sequence

import numpy as np

from . import _lib
from .dataset import Dataset, SubDataset
from .device import get_context
from .node import Node, TreeBatch, flatten_trees


def _as_batch(trees, dtype) -> TreeBatch:
    if isinstance(trees, TreeBatch):
        return trees if trees.val.dtype == dtype else trees.astype(dtype)
    if isinstance(trees, Node) or hasattr(trees, "tree"):
        trees = [trees]
    return flatten_trees(trees, dtype=dtype)


def eval_loss_batch(trees, dataset, options, *, ctx=None):
    """Loss of every tree on ``dataset`` (Dataset or SubDataset) -> (losses[T], complete[bool]).

    Per tree this is ``_eval_loss`` (src/LossFunctions.jl:90-117): ``L(Inf)`` when the evaluation
    is incomplete, else the (weighted) mean elementwise loss.  Custom ``loss_function`` /
    ``loss_function_expression`` objectives are Julia functions and stay on the caller's CPU path.
    """
    if options.loss_function is not None or options.loss_function_expression is not None:
        raise NotImplementedError("custom objectives are evaluated by the reference CPU path")
    ctx = ctx or get_context()
    full = dataset.full
    tb = _as_batch(trees, full.dtype)
    nt = tb.n_trees
    losses = np.empty(nt, dtype=full.dtype)
    complete = np.empty(nt, dtype=np.uint8)
    if full.y is None:
        raise ValueError("dataset has no y")
    idx = dataset.indices
    s = tb.to_struct()
    _lib.check(
        _lib.lib.sr_eval_loss_batch(
            ctx.handle,
            full.device_handle(ctx),
            ctx.opset_id(options.operators),
            ctypes.byref(s),
            None if idx is None else idx.ctypes.data_as(ctypes.c_void_p),
            0 if idx is None else int(idx.size),
            ctx.loss_code(options),
            losses.ctypes.data_as(ctypes.c_void_p),
            complete.ctypes.data_as(ctypes.c_void_p),
        )
    )
    return losses, complete.astype(bool)


def _views(tree_view, view_rows, nt):
    tv = np.ascontiguousarray(tree_view, dtype=np.int32)
    vr = np.ascontiguousarray(view_rows, dtype=np.int64)
    if vr.ndim != 2 or tv.shape != (nt,):
        raise ValueError("view_rows must be [n_views, view_len] and tree_view one view per tree")
    return tv, vr


def eval_loss_batch_views(trees, dataset, options, tree_view, view_rows, *, ctx=None):
    """``eval_loss_batch`` with tree t on the rows ``view_rows[tree_view[t]]`` of ``dataset`` (a Dataset):
    every island's trees on its own minibatch (src/SingleIteration.jl:40) in ONE device call."""
    ctx = ctx or get_context()
    full = dataset.full
    tb = _as_batch(trees, full.dtype)
    nt = tb.n_trees
    tv, vr = _views(tree_view, view_rows, nt)
    losses = np.empty(nt, dtype=full.dtype)
    complete = np.empty(nt, dtype=np.uint8)
    s = tb.to_struct()
    p = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    _lib.check(_lib.lib.sr_eval_loss_batch_views(
        ctx.handle, full.device_handle(ctx), ctx.opset_id(options.operators), ctypes.byref(s), p(tv), int(vr.shape[0]),
        p(vr), int(vr.shape[1]), ctx.loss_code(options), p(losses), p(complete)))
    return losses, complete.astype(bool)


def eval_grad_batch_views(trees, dataset, options, tree_view, view_rows, *, ctx=None):
    """``eval_grad_batch`` over several row views in one call (as ``eval_loss_batch_views``)."""
    ctx = ctx or get_context()
    full = dataset.full
    tb = _as_batch(trees, full.dtype)
    nt = tb.n_trees
    tv, vr = _views(tree_view, view_rows, nt)
    losses = np.empty(nt, dtype=full.dtype)
    complete = np.empty(nt, dtype=np.uint8)
    grads = np.zeros(int(tb.constant_mask().sum()) + 1, dtype=full.dtype)
    s = tb.to_struct()
    p = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    _lib.check(_lib.lib.sr_eval_grad_batch_views(
        ctx.handle, full.device_handle(ctx), ctx.opset_id(options.operators), ctypes.byref(s), p(tv), int(vr.shape[0]),
        p(vr), int(vr.shape[1]), ctx.loss_code(options), p(losses), p(grads), p(complete)))
    return losses, grads[:-1], complete.astype(bool)


def eval_grad_batch(trees, dataset, options, *, ctx=None):
    """Loss and its gradient with respect to every tree's constants, for a whole batch.

    Returns ``(losses[T], grads[T], complete[bool])``; ``grads`` holds each tree's constants in
    pre-order (``get_scalar_constants``) at ``TreeBatch.constant_offsets()``.  This is the
    objective/gradient pair of reference src/ConstantOptimization.jl:126-167 (``Evaluator`` /
    ``GradEvaluator`` with a forward-mode backend) computed on the device by forward-mode dual
    numbers; an incomplete tree has loss ``Inf`` and a zero gradient (``eval_loss`` is the
    constant ``L(Inf)`` there).
    """
    if options.loss_function is not None or options.loss_function_expression is not None:
        raise NotImplementedError("custom objectives are evaluated by the reference CPU path")
    ctx = ctx or get_context()
    full = dataset.full
    tb = _as_batch(trees, full.dtype)
    nt = tb.n_trees
    losses = np.empty(nt, dtype=full.dtype)
    complete = np.empty(nt, dtype=np.uint8)
    grads = np.zeros(int(tb.constant_mask().sum()) + 1, dtype=full.dtype)
    idx = dataset.indices
    s = tb.to_struct()
    _lib.check(
        _lib.lib.sr_eval_grad_batch(
            ctx.handle,
            full.device_handle(ctx),
            ctx.opset_id(options.operators),
            ctypes.byref(s),
            None if idx is None else idx.ctypes.data_as(ctypes.c_void_p),
            0 if idx is None else int(idx.size),
            ctx.loss_code(options),
            losses.ctypes.data_as(ctypes.c_void_p),
            grads.ctypes.data_as(ctypes.c_void_p),
            complete.ctypes.data_as(ctypes.c_void_p),
        )
    )
    return losses, grads[:-1], complete.astype(bool)


def eval_tree_array_batch(trees, dataset, options, *, ctx=None):
    """Predictions of every tree: (out[n_trees, n_rows], complete[n_trees])."""
    ctx = ctx or get_context()
    full = dataset.full
    tb = _as_batch(trees, full.dtype)
    idx = dataset.indices
    n_rows = full.n if idx is None else int(idx.size)
    out = np.empty((tb.n_trees, n_rows), dtype=full.dtype)
    complete = np.empty(tb.n_trees, dtype=np.uint8)
    s = tb.to_struct()
    _lib.check(
        _lib.lib.sr_eval_tree_array(
            ctx.handle,
            full.device_handle(ctx),
            ctx.opset_id(options.operators),
            ctypes.byref(s),
            None if idx is None else idx.ctypes.data_as(ctypes.c_void_p),
            0 if idx is None else int(idx.size),
            out.ctypes.data_as(ctypes.c_void_p),
            complete.ctypes.data_as(ctypes.c_void_p),
        )
    )
    return out, complete.astype(bool)


def eval_tree_array(tree, X, options):
    """``eval_tree_array(tree, X, options) -> (output, complete)``
    (src/InterfaceDynamicExpressions.jl:58-88).  ``X`` is ``[nfeatures, n]`` or a Dataset."""
    if isinstance(X, (Dataset, SubDataset)):
        out, comp = eval_tree_array_batch([tree], X, options)
        return out[0], bool(comp[0])
    ds = Dataset(np.asarray(X))
    try:
        out, comp = eval_tree_array_batch([tree], ds, options)
    finally:
        ds.free_device()
    return out[0], bool(comp[0])


def dimensional_regularization(tree, dataset, options):
    # violates_dimensional_constraints is `false` without units (src/DimensionalAnalysis.jl:267-275)
    return dataset.full.dtype.type(0)


def eval_loss(tree, dataset, options, *, regularization: bool = True, idx=None):
    """``eval_loss`` (src/LossFunctions.jl:139-159) for one tree."""
    if idx is not None:
        dataset = SubDataset(dataset.full, idx)
    losses, _ = eval_loss_batch([tree], dataset, options)
    loss = losses[0]
    if regularization:
        loss = loss + dimensional_regularization(tree, dataset, options)
    return loss


def compute_complexity(tree, options=None) -> int:
    """Default complexity = number of nodes (src/Complexity.jl:29-41)."""
    t = getattr(tree, "tree", tree)
    return t.count_nodes()


def loss_to_cost(loss, use_baseline: bool, baseline, member, options, complexity=None):
    """src/LossFunctions.jl:170-190: loss / normalization + L(size * parsimony::Float32)."""
    L = type(loss) if isinstance(loss, np.floating) else np.float64
    normalization = baseline if (baseline >= L(0.01) and use_baseline) else L(0.01)
    loss_val = L(loss) / L(normalization)
    size = complexity if complexity is not None else compute_complexity(member, options)
    parsimony_term = np.float32(size) * np.float32(options.parsimony)
    return L(loss_val + L(parsimony_term))


def eval_cost(dataset, member, options, *, complexity=None):
    """``eval_cost`` (src/LossFunctions.jl:193-209) -> (cost, loss)."""
    tree = getattr(member, "tree", member)
    result_loss = eval_loss(tree, dataset, options)
    cost = loss_to_cost(result_loss, dataset.use_baseline, dataset.baseline_loss, member, options, complexity)
    return cost, result_loss


def eval_cost_batch(members: Sequence, dataset, options, *, complexities=None):
    """Batched ``eval_cost`` for a population: one device launch for all members."""
    trees = [getattr(m, "tree", m) for m in members]
    losses, _ = eval_loss_batch(trees, dataset, options)
    if complexities is None:
        complexities = [compute_complexity(t) for t in trees]
    costs = np.array(
        [
            loss_to_cost(losses[i], dataset.use_baseline, dataset.baseline_loss, trees[i], options, complexities[i])
            for i in range(len(trees))
        ],
        dtype=losses.dtype,
    )
    return costs, losses


def update_baseline_loss_(dataset, options):
    """``update_baseline_loss!`` (src/LossFunctions.jl:219-234): loss of the constant-0 tree."""
    T = dataset.full.dtype.type
    example_tree = Node(val=T(0))
    baseline_loss = eval_loss(example_tree, dataset, options)
    if np.isfinite(baseline_loss):
        dataset.baseline_loss = baseline_loss
        dataset.use_baseline = True
    else:
        dataset.baseline_loss = T(1)
        dataset.use_baseline = False
    return None


score_func = eval_cost  # deprecated alias kept by the reference (src/LossFunctions.jl:212)
