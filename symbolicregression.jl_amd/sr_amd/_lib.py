"""ctypes binding of the C ABI in ``include/sr_amd.h`` (``lib/libsr_amd.so``).

This is the same binding a Julia ``ccall`` wrapper makes; Python uses it for the
host-side mirror of SymbolicRegression's scoring API and for the tests / benchmark.  There is no
fallback: if the shared library is missing the import fails loudly.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_char_p, c_double, c_int, c_int64, c_uint8, c_uint16, c_uint32, c_void_p

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get(
    "SR_AMD_LIB", os.path.join(os.path.dirname(_HERE), "lib", "libsr_amd.so")
)

SR_OK = 0
SR_ERR_INVALID_ARG = -1
SR_ERR_HIP = -2
SR_ERR_UNSUPPORTED_OP = -3
SR_ERR_BAD_TREE = -4
SR_ERR_TOO_DEEP = -5
SR_ERR_NO_DEVICE = -6

SR_DTYPE_F32 = 0
SR_DTYPE_F64 = 1
SR_LOSS_L2DIST = 0
SR_LOSS_L1DIST = 1

SR_FLAG_NONFINITE = 1
SR_FLAG_BIG = 2
SR_FLAG_STATIC = 4
SR_FLAG_ELEMINF = 8

# Every symbol include/sr_amd.h declares (checked by tests/test_abi.py).
EXPORTED_SYMBOLS = (
    "sr_last_error",
    "sr_version",
    "sr_device_count",
    "sr_init",
    "sr_shutdown",
    "sr_register_opset",
    "sr_register_loss",
    "sr_dataset_upload",
    "sr_dataset_free",
    "sr_dataset_info",
    "sr_eval_loss_batch",
    "sr_eval_loss_batch_views",
    "sr_eval_tree_array",
    "sr_eval_loss_partials",
    "sr_eval_loss_partials_packed",
    "sr_comm_unique_id",
    "sr_comm_init",
    "sr_comm_init_host",
    "sr_comm_destroy",
    "sr_eval_loss_partials_allreduce",
    "sr_eval_loss_sharded",
    "sr_eval_loss_tree_sharded",
    "sr_comm_info",
    "sr_runtime_info",
    "sr_max_checks",
    "sr_jsum_range_count",
    "sr_jsum_ranges",
    "sr_jsum_partials",
    "sr_jsum_finite",
    "sr_finalize_losses",
    "sr_dataset_denominator",
    "sr_eval_grad_batch",
    "sr_eval_grad_batch_views",
    "sr_compile_info",
    "sr_host_unary",
    "sr_last_kernel_ms",
    "sr_last_phase_ms",
    "sr_set_tuning",
    "sr_tuning_info",
    "sr_ref_fold_info",
    "sr_last_grad_info",
    "sr_search_create",
    "sr_search_free",
    "sr_search_use_device",
    "sr_search_add_device",
    "sr_search_use_callbacks",
    "sr_search_start",
    "sr_search_iterate",
    "sr_search_head",
    "sr_search_export",
    "sr_search_import",
    "sr_search_get_info",
    "sr_search_member_count",
    "sr_search_members",
    "sr_optimize_constants_batch",
    "sr_gen_random_population",
    "sr_optimize_constants_callbacks",
)

# mutation kinds in sr_search_options.mutation_weights order (SR_MUT_*)
MUTATIONS = ("mutate_constant", "mutate_operator", "mutate_feature", "swap_operands", "rotate_tree", "add_node",
             "insert_node", "delete_node", "simplify", "randomize", "do_nothing", "optimize")
SR_SEARCH_HALL_OF_FAME = -1
SR_SEARCH_PARETO = -2


class SRError(RuntimeError):
    """Error returned by libsr_amd (status code + sr_last_error message)."""

    def __init__(self, code: int, msg: str):
        super().__init__(f"libsr_amd error {code}: {msg}")
        self.code = code


class UnsupportedOperatorError(SRError):
    pass


class SrTreeBatch(ctypes.Structure):
    _fields_ = [
        ("n_trees", c_int64),
        ("offsets", POINTER(c_int64)),
        ("degree", POINTER(c_uint8)),
        ("op", POINTER(c_uint8)),
        ("feature", POINTER(c_uint16)),
        ("constant", POINTER(c_uint8)),
        ("val", c_void_p),
    ]


c_float = ctypes.c_float


class SrSearchOptions(ctypes.Structure):
    _fields_ = [
        ("populations", c_int), ("population_size", c_int), ("ncycles_per_iteration", c_int),
        ("tournament_selection_n", c_int), ("tournament_selection_p", c_float),
        ("maxsize", c_int), ("maxdepth", c_int), ("parsimony", c_float), ("crossover_probability", c_float),
        ("annealing", c_int), ("alpha", c_float), ("perturbation_factor", c_float),
        ("probability_negate_constant", c_float), ("use_frequency", c_int), ("use_frequency_in_tournament", c_int),
        ("adaptive_parsimony_scaling", c_double), ("fraction_replaced", c_float), ("fraction_replaced_hof", c_float),
        ("topn", c_int), ("migration", c_int), ("hof_migration", c_int), ("skip_mutation_failures", c_int),
        ("should_simplify", c_int), ("should_optimize_constants", c_int), ("optimizer_probability", c_float),
        ("optimizer_iterations", c_int), ("optimizer_nrestarts", c_int), ("batching", c_int),
        ("batch_size", c_int64), ("warmup_maxsize_by", c_float), ("mutation_weights", c_double * len(MUTATIONS)),
        ("optimizer_f_calls_limit", c_int64),
    ]


class SrSearchInfo(ctypes.Structure):
    _fields_ = [
        ("iterations", c_int64), ("s_r_cycles", c_int64), ("device_calls", c_int64), ("num_evals", c_double),
        ("device_ms", c_double), ("host_ms", c_double), ("baseline_loss", c_double), ("use_baseline", c_int),
        ("kernel_ms", c_double),
    ]


# CPU scorer callbacks (tests): sr_loss_fn / sr_grad_fn
LOSS_FN = ctypes.CFUNCTYPE(c_int, c_void_p, POINTER(SrTreeBatch), c_void_p, c_int64, c_void_p, c_void_p)
GRAD_FN = ctypes.CFUNCTYPE(c_int, c_void_p, POINTER(SrTreeBatch), c_void_p, c_int64, c_void_p, c_void_p, c_void_p)
# host collectives of sr_comm_init_host: sr_host_allreduce_fn / sr_host_allgather_fn
HOST_ALLREDUCE_FN = ctypes.CFUNCTYPE(c_int, c_void_p, POINTER(c_double), c_int64)
HOST_ALLGATHER_FN = ctypes.CFUNCTYPE(c_int, c_void_p, c_void_p, c_void_p, c_int64)


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"libsr_amd.so not found at {LIB_PATH}: build it with `make -C symbolicregression.jl_amd` "
            "(or __graft_entry__.build()); there is no CPU fallback for the device path"
        )
    lib = ctypes.CDLL(LIB_PATH)
    P = c_void_p
    proto = {
        "sr_last_error": (c_char_p, []),
        "sr_version": (c_int, []),
        "sr_device_count": (c_int, [POINTER(c_int)]),
        "sr_init": (c_int, [c_int, POINTER(P)]),
        "sr_shutdown": (c_int, [P]),
        "sr_register_opset": (
            c_int,
            [P, c_int, POINTER(c_char_p), c_int, POINTER(c_char_p), POINTER(c_int)],
        ),
        "sr_register_loss": (c_int, [P, c_int, c_double, POINTER(c_int)]),
        "sr_dataset_upload": (c_int, [P, c_int, P, c_int64, c_int64, P, P, POINTER(P)]),
        "sr_dataset_free": (c_int, [P]),
        "sr_dataset_info": (c_int, [P, POINTER(c_int), POINTER(c_int64), POINTER(c_int64)]),
        "sr_eval_loss_batch": (
            c_int,
            [P, P, c_int, POINTER(SrTreeBatch), P, c_int64, c_int, P, P],
        ),
        "sr_eval_loss_batch_views": (
            c_int,
            [P, P, c_int, POINTER(SrTreeBatch), P, c_int, P, c_int64, c_int, P, P],
        ),
        "sr_eval_grad_batch_views": (
            c_int,
            [P, P, c_int, POINTER(SrTreeBatch), P, c_int, P, c_int64, c_int, P, P, P],
        ),
        "sr_eval_tree_array": (c_int, [P, P, c_int, POINTER(SrTreeBatch), P, c_int64, P, P]),
        "sr_eval_loss_partials": (
            c_int,
            [P, P, c_int, POINTER(SrTreeBatch), c_int64, c_int, P, P, c_int],
        ),
        "sr_max_checks": (c_int, [P, c_int, c_int, POINTER(SrTreeBatch), POINTER(c_int)]),
        "sr_comm_unique_id": (c_int, [P]),
        "sr_comm_init": (c_int, [P, c_int, c_int, P]),
        "sr_comm_init_host": (c_int, [P, c_int, c_int, HOST_ALLREDUCE_FN, HOST_ALLGATHER_FN, P]),
        "sr_comm_destroy": (c_int, [P]),
        "sr_eval_loss_partials_allreduce": (c_int, [P, P, c_int, POINTER(SrTreeBatch), c_int64, c_int, P]),
        "sr_eval_loss_sharded": (c_int, [P, P, c_int, POINTER(SrTreeBatch), c_int, P, P]),
        "sr_eval_loss_tree_sharded": (c_int, [P, P, c_int, POINTER(SrTreeBatch), c_int, P, P]),
        "sr_comm_info": (c_int, [P, POINTER(c_int), POINTER(c_int), c_char_p, c_int64]),
        "sr_runtime_info": (c_int, [c_char_p, c_int64]),
        "sr_eval_loss_partials_packed": (
            c_int,
            [P, P, c_int, POINTER(SrTreeBatch), c_int64, c_int, P, c_int],
        ),
        "sr_jsum_range_count": (c_int, [c_int64, c_int64, c_int64, POINTER(c_int64)]),
        "sr_jsum_ranges": (c_int, [c_int64, c_int64, c_int64, P, P, P, P]),
        "sr_jsum_partials": (
            c_int,
            [P, P, c_int, POINTER(SrTreeBatch), P, c_int64, c_int, c_int64, c_int64, P],
        ),
        "sr_jsum_finite": (c_int, [c_int, c_int64, c_int, P, P, c_int64, P]),
        "sr_finalize_losses": (
            c_int,
            [c_int, c_int64, P, P, c_double, P, c_int64, P, P, P],
        ),
        "sr_dataset_denominator": (c_int, [P, POINTER(c_double)]),
        "sr_eval_grad_batch": (
            c_int,
            [P, P, c_int, POINTER(SrTreeBatch), P, c_int64, c_int, P, P, P],
        ),
        "sr_compile_info": (
            c_int,
            [c_int, c_int, POINTER(c_char_p), c_int, POINTER(c_char_p), POINTER(SrTreeBatch), c_int64,
             c_int64, P, P, POINTER(c_int), P, c_int64],
        ),
        "sr_host_unary": (c_int, [c_int, c_char_p, c_int64, P, P]),
        "sr_last_kernel_ms": (c_int, [P, POINTER(c_double), POINTER(c_double)]),
        "sr_last_phase_ms": (c_int, [P, POINTER(c_double), c_int]),
        "sr_set_tuning": (c_int, [P, ctypes.c_char_p, ctypes.c_int64]),
        "sr_tuning_info": (c_int, [P, POINTER(c_int), POINTER(c_int64)]),
        "sr_ref_fold_info": (c_int, [P, POINTER(c_int), POINTER(c_int64), POINTER(c_int64), POINTER(c_double)]),
        "sr_last_grad_info": (c_int, [P, c_int, P, P, P, P]),
        "sr_search_create": (
            c_int,
            [c_int, c_int64, c_int64, c_int, POINTER(c_char_p), c_int, POINTER(c_char_p), POINTER(SrSearchOptions),
             ctypes.c_uint64, c_int, c_int, POINTER(P)],
        ),
        "sr_search_free": (c_int, [P]),
        "sr_search_use_device": (c_int, [P, P, P, c_int, c_int]),
        "sr_search_add_device": (c_int, [P, P, P, c_int, c_int]),
        "sr_search_use_callbacks": (c_int, [P, LOSS_FN, GRAD_FN, P]),
        "sr_search_start": (c_int, [P, c_int]),
        "sr_search_iterate": (c_int, [P]),
        "sr_search_head": (c_int, [P]),
        "sr_search_export": (c_int, [P, P, c_int64, POINTER(c_int64)]),
        "sr_search_import": (c_int, [P, P, c_int64]),
        "sr_search_get_info": (c_int, [P, POINTER(SrSearchInfo)]),
        "sr_search_member_count": (c_int, [P, c_int, POINTER(c_int64), POINTER(c_int64)]),
        "sr_search_members": (c_int, [P, c_int, P, P, P, P, P, P, P, P, P, P, P, P]),
        "sr_optimize_constants_callbacks": (
            c_int,
            [c_int, POINTER(SrTreeBatch), P, c_int64, c_int, c_int64, c_int, ctypes.c_uint64, LOSS_FN, GRAD_FN, P, P, P,
             P, P],
        ),
        "sr_gen_random_population": (
            c_int,
            [c_int, c_int64, c_int64, c_int, c_int, c_int, ctypes.c_uint64, c_int64, P, P, P, P, P, P],
        ),
        "sr_optimize_constants_batch": (
            c_int,
            [P, P, c_int, POINTER(SrTreeBatch), P, c_int64, c_int, c_int, c_int64, c_int, ctypes.c_uint64, P, P, P, P],
        ),
    }
    for name, (res, args) in proto.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


lib = _load()


def last_error() -> str:
    msg = lib.sr_last_error()
    return msg.decode() if msg else ""


def check(rc: int) -> None:
    if rc == SR_OK:
        return
    msg = last_error()
    if rc == SR_ERR_UNSUPPORTED_OP:
        raise UnsupportedOperatorError(rc, msg)
    raise SRError(rc, msg)


def runtime_info() -> dict:
    """{"hip": file, "rccl": file}: the HIP runtime and RCCL the library's calls bind to (no device needed)."""
    buf = ctypes.create_string_buffer(4096)
    check(lib.sr_runtime_info(buf, len(buf)))
    return dict(kv.split("=", 1) for kv in buf.value.decode().split(";") if "=" in kv)


def device_count() -> int:
    c = c_int(0)
    rc = lib.sr_device_count(ctypes.byref(c))
    if rc != SR_OK:
        return 0
    return int(c.value)
