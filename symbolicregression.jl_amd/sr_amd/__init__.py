"""sr_amd — MI355X-native scoring path of SymbolicRegression.jl (host-side mirror of its API).

Public names follow the reference: ``Options``, ``Dataset``, ``batch``, ``Node``,
``eval_tree_array``, ``eval_loss``, ``eval_cost``, ``loss_to_cost``, ``update_baseline_loss_``
(Julia ``update_baseline_loss!``), plus the batched ``eval_loss_batch`` / ``eval_cost_batch`` that
score a whole population in one device launch.  All evaluation runs in ``libsr_amd.so`` on the GPU.
"""
from . import _lib
from ._lib import SRError, UnsupportedOperatorError
from .constant_optimization import optimize_constants_batch
from .dataset import Dataset, SubDataset, batch
from .device import DeviceContext, device_available, get_context
from .loss import (
    compute_complexity,
    eval_cost,
    eval_cost_batch,
    eval_grad_batch,
    eval_grad_batch_views,
    eval_loss,
    eval_loss_batch,
    eval_loss_batch_views,
    eval_tree_array,
    eval_tree_array_batch,
    loss_to_cost,
    score_func,
    update_baseline_loss_,
)
from .mutation import gen_random_batch, gen_random_population, gen_random_tree_fixed_size, make_random_leaf
from .node import (
    Node,
    TreeBatch,
    apply_binary,
    apply_unary,
    extend_operators,
    flatten_trees,
    get_scalar_constants,
    parse_expression,
    set_scalar_constants,
    string_tree,
)
from .operators import OperatorEnum
from .options import Options
from .search import HallOfFame, PopMember, SearchOptions, equation_search

__all__ = [
    "Options", "OperatorEnum", "Dataset", "SubDataset", "batch", "Node", "TreeBatch", "flatten_trees",
    "extend_operators", "apply_unary", "apply_binary", "parse_expression", "string_tree",
    "get_scalar_constants", "set_scalar_constants", "eval_tree_array", "eval_tree_array_batch",
    "eval_loss", "eval_loss_batch", "eval_grad_batch", "eval_loss_batch_views", "eval_grad_batch_views", "eval_cost", "eval_cost_batch", "loss_to_cost",
    "update_baseline_loss_", "score_func", "compute_complexity", "gen_random_tree_fixed_size",
    "gen_random_population", "gen_random_batch", "make_random_leaf", "get_context", "device_available", "DeviceContext",
    "SRError", "UnsupportedOperatorError", "optimize_constants_batch", "equation_search", "SearchOptions",
    "PopMember", "HallOfFame",
]
