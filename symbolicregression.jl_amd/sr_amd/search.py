"""``equation_search`` on the native search engine (§8(a) A9, A10).

The search loop itself is C++ (``csrc/sr_search.cpp``, C ABI ``sr_search_*``): ``s_r_cycle`` /
``reg_evol_cycle`` / ``next_generation`` / ``crossover_generation``, ``optimize_and_simplify_population``
and the head's per-island bookkeeping (src/SingleIteration.jl, src/RegularizedEvolution.jl,
src/Mutate.jl, src/MutationFunctions.jl, src/Population.jl, src/SymbolicRegression.jl:1040-1140).
This module is the reference-shaped API around it: options in, ``PopMember`` / ``HallOfFame``
results out, and the island exchange between ranks for ``distributed=True``.

MI355X-first change: islands advance in LOCK-STEP — at every regularised-evolution round the
children of ALL islands are scored by ONE batched device call (each island's serial semantics are
kept), and constant optimisation runs batched over every island's selected members.  Random streams
and birth counters are per island (csrc/sr_rng.h), so trajectories are reproducible from ``seed``
(not equal to a Julia run's), and an island-sharded search equals the single-process one.
"""
from __future__ import annotations

import ctypes
import time
from dataclasses import dataclass, field

import numpy as np

from . import _lib
from .dataset import Dataset
from .node import TreeBatch

MUTATIONS = _lib.MUTATIONS

# v1 defaults (src/Options.jl:1174-1188); form/break_connection are 0 for plain Node trees
DEFAULT_MUTATION_WEIGHTS = dict(mutate_constant=0.0346, mutate_operator=0.293, mutate_feature=0.1,
                                swap_operands=0.198, rotate_tree=4.26, add_node=2.47, insert_node=0.0112,
                                delete_node=0.870, simplify=0.00209, randomize=0.000502, do_nothing=0.273,
                                optimize=0.0)


@dataclass
class SearchOptions:
    """Search knobs with the reference's v1 defaults (src/Options.jl:1161-1208).  ``should_simplify``
    defaults to True as the reference's does without custom losses or constraints (src/Options.jl:813-821)."""
    crossover_probability: float = 0.0259
    annealing: bool = True
    alpha: float = 3.17
    perturbation_factor: float = 0.129
    probability_negate_constant: float = 0.00743
    use_frequency: bool = True
    use_frequency_in_tournament: bool = True
    adaptive_parsimony_scaling: float = 1040.0
    fraction_replaced: float = 0.00036
    fraction_replaced_hof: float = 0.0614
    topn: int = 12
    migration: bool = True
    hof_migration: bool = True
    skip_mutation_failures: bool = True
    should_simplify: bool = True
    warmup_maxsize_by: float = 0.0
    mutation_weights: dict = field(default_factory=lambda: dict(DEFAULT_MUTATION_WEIGHTS))


class PopMember:
    """src/PopMember.jl: tree, cost, loss, birth order, complexity, ref / parent."""
    __slots__ = ("tree", "cost", "loss", "birth", "complexity", "ref", "parent")

    def __init__(self, tree, cost, loss, complexity, parent=-1, birth=0, ref=0):
        self.tree = tree
        self.cost = cost
        self.loss = loss
        self.complexity = int(complexity)
        self.birth = int(birth)
        self.ref = int(ref)
        self.parent = int(parent)

    def copy(self):
        return PopMember(self.tree.copy(), self.cost, self.loss, self.complexity, self.parent, self.birth, self.ref)


class HallOfFame:
    """Best member per complexity (src/HallOfFame.jl)."""

    def __init__(self, maxsize):
        self.members = [None] * maxsize
        self.exists = [False] * maxsize

    def pareto_frontier(self):
        """calculate_pareto_frontier (src/HallOfFame.jl:96-124): kept unless some existing simpler
        member's loss is <= its loss."""
        out = []
        for size in range(len(self.members)):
            if not self.exists[size]:
                continue
            m = self.members[size]
            if not any(self.exists[i] and m.loss >= self.members[i].loss for i in range(size)):
                out.append(m.copy())
        return out


@dataclass
class SearchResult:
    hall_of_fame: HallOfFame
    pareto_frontier: list
    populations: list
    iterations: int
    wall_s: float
    s_r_cycles: int
    num_evals: float
    device_calls: int
    device_s: float = 0.0
    host_s: float = 0.0
    kernel_s: float = 0.0  # device-busy time of the scoring launches (interpreter), inside device_s


def make_callbacks(dtype, loss_fn, grad_fn=None):
    """(sr_loss_fn, sr_grad_fn) ctypes callbacks around Python scorers: loss_fn(TreeBatch, rows or None)
    -> losses (Inf where incomplete); grad_fn(TreeBatch, rows) -> (losses, gradients over the batch's
    constants).  Keep the returned objects alive while the library may call them."""
    dtype = np.dtype(dtype)

    def batch_of(p):
        s = p.contents
        nt = int(s.n_trees)
        offs = np.ctypeslib.as_array(s.offsets, shape=(nt + 1,)).copy()
        nn = int(offs[-1])

        def arr(ptr, t):
            return np.ctypeslib.as_array(ptr, shape=(nn,)).copy() if nn else np.zeros(0, t)
        val = np.ctypeslib.as_array(ctypes.cast(s.val, ctypes.POINTER(
            ctypes.c_float if dtype == np.float32 else ctypes.c_double)), shape=(nn,)).copy()
        return TreeBatch(offs, arr(s.degree, np.uint8), arr(s.op, np.uint8), arr(s.feature, np.uint16),
                         arr(s.constant, np.uint8), val)

    def rows_of(p, n):
        if not p or n <= 0:
            return None
        return np.ctypeslib.as_array(ctypes.cast(p, ctypes.POINTER(ctypes.c_int64)), shape=(n,)).copy()

    def out_arr(p, n, t):
        return np.ctypeslib.as_array(ctypes.cast(p, ctypes.POINTER(t)), shape=(n,))

    ct = ctypes.c_float if dtype == np.float32 else ctypes.c_double

    def loss_cb(user, trees, rows, n_idx, out_loss, out_complete):
        try:
            tb = batch_of(trees)
            losses = np.asarray(loss_fn(tb, rows_of(rows, n_idx)), dtype=dtype)
            out_arr(out_loss, tb.n_trees, ct)[:] = losses
            out_arr(out_complete, tb.n_trees, ctypes.c_uint8)[:] = np.isfinite(losses)
            return 0
        except Exception:  # pragma: no cover - surfaced as an error code
            import traceback
            traceback.print_exc()
            return _lib.SR_ERR_INVALID_ARG

    def grad_cb(user, trees, rows, n_idx, out_loss, out_grad, out_complete):
        try:
            tb = batch_of(trees)
            losses, g = grad_fn(tb, rows_of(rows, n_idx))
            losses = np.asarray(losses, dtype=dtype)
            out_arr(out_loss, tb.n_trees, ct)[:] = losses
            nc = int(np.count_nonzero(tb.constant_mask()))
            if nc:
                out_arr(out_grad, nc, ct)[:] = np.asarray(g, dtype=dtype)
            out_arr(out_complete, tb.n_trees, ctypes.c_uint8)[:] = np.isfinite(losses)
            return 0
        except Exception:  # pragma: no cover
            import traceback
            traceback.print_exc()
            return _lib.SR_ERR_INVALID_ARG

    return _lib.LOSS_FN(loss_cb), (_lib.GRAD_FN(grad_cb) if grad_fn else _lib.GRAD_FN())


def search_options_struct(options, so: SearchOptions) -> _lib.SrSearchOptions:
    """Options + SearchOptions -> sr_search_options (Float32 fields as the reference stores them)."""
    o = _lib.SrSearchOptions()
    o.populations = int(options.populations)
    o.population_size = int(options.population_size)
    o.ncycles_per_iteration = int(options.ncycles_per_iteration)
    o.tournament_selection_n = int(options.tournament_selection_n)
    o.tournament_selection_p = float(options.tournament_selection_p)
    o.maxsize = int(options.maxsize)
    o.maxdepth = int(options.maxdepth)
    o.parsimony = float(options.parsimony)
    o.crossover_probability = float(so.crossover_probability)
    o.annealing = int(bool(so.annealing))
    o.alpha = float(so.alpha)
    o.perturbation_factor = float(so.perturbation_factor)
    o.probability_negate_constant = float(so.probability_negate_constant)
    o.use_frequency = int(bool(so.use_frequency))
    o.use_frequency_in_tournament = int(bool(so.use_frequency_in_tournament))
    o.adaptive_parsimony_scaling = float(so.adaptive_parsimony_scaling)
    o.fraction_replaced = float(so.fraction_replaced)
    o.fraction_replaced_hof = float(so.fraction_replaced_hof)
    o.topn = int(so.topn)
    o.migration = int(bool(so.migration))
    o.hof_migration = int(bool(so.hof_migration))
    o.skip_mutation_failures = int(bool(so.skip_mutation_failures))
    o.should_simplify = int(bool(so.should_simplify))
    o.should_optimize_constants = int(bool(options.should_optimize_constants))
    o.optimizer_probability = float(options.optimizer_probability)
    o.optimizer_iterations = int(options.optimizer_iterations)
    o.optimizer_nrestarts = int(options.optimizer_nrestarts)
    o.optimizer_f_calls_limit = int(options.optimizer_f_calls_limit)
    if options.should_optimize_constants and getattr(options, "optimizer_algorithm", "BFGS") != "BFGS":
        raise NotImplementedError(f"optimizer_algorithm={options.optimizer_algorithm!r}: the native search runs the "
                                  "device BFGS optimiser only; the reference's CPU search is the path for it")
    o.batching = int(bool(options.batching))
    o.batch_size = int(options.batch_size)
    o.warmup_maxsize_by = float(so.warmup_maxsize_by)
    unknown = set(so.mutation_weights) - set(MUTATIONS)
    if unknown:
        raise ValueError(f"unknown mutation weights {sorted(unknown)}")
    for k, name in enumerate(MUTATIONS):
        o.mutation_weights[k] = float(so.mutation_weights.get(name, 0.0))
    return o


def _names(seq):
    arr = (ctypes.c_char_p * max(1, len(seq)))(*[s.encode() for s in seq])
    return arr


class NativeSearch:
    """Owner of one ``sr_search`` handle (islands of this rank, head state, scorer)."""

    def __init__(self, dataset, options, so, seed, rank=0, world=1):
        self.dtype = dataset.dtype
        self.options = options
        ops = options.operators
        unary, binary = list(ops.unaops), list(ops.binops)
        self._un, self._bn = _names(unary), _names(binary)
        self._opts = search_options_struct(options, so)
        h = ctypes.c_void_p()
        dt = _lib.SR_DTYPE_F32 if self.dtype == np.float32 else _lib.SR_DTYPE_F64
        _lib.check(_lib.lib.sr_search_create(dt, int(dataset.nfeatures), int(dataset.n), len(unary), self._un,
                                             len(binary), self._bn, ctypes.byref(self._opts),
                                             int(seed) & 0xFFFFFFFFFFFFFFFF, int(rank), int(world), ctypes.byref(h)))
        self.h = h
        self._keep = []

    def __del__(self):
        h = getattr(self, "h", None)
        if h is not None and h.value:
            _lib.lib.sr_search_free(h)
            self.h = None

    def use_device(self, dataset, ctx=None):
        from .device import get_context

        ctx = ctx or get_context()
        self._keep.append(dataset)
        _lib.check(_lib.lib.sr_search_use_device(self.h, ctx.handle, dataset.device_handle(ctx),
                                                 ctx.opset_id(self.options.operators), ctx.loss_code(self.options)))

    def add_device(self, dataset, ctx):
        """An extra scoring lane (its own context and dataset copy): iterate() splits this rank's
        islands over the lanes, one host thread each."""
        self._keep.append(dataset)
        _lib.check(_lib.lib.sr_search_add_device(self.h, ctx.handle, dataset.device_handle(ctx),
                                                 ctx.opset_id(self.options.operators), ctx.loss_code(self.options)))

    def use_callbacks(self, loss_fn, grad_fn=None):
        """CPU scorers (tests): loss_fn(TreeBatch, rows or None) -> losses (Inf where incomplete);
        grad_fn(TreeBatch, rows) -> (losses, gradients over the batch's constants)."""
        self._cbs = make_callbacks(self.dtype, loss_fn, grad_fn)
        _lib.check(_lib.lib.sr_search_use_callbacks(self.h, self._cbs[0], self._cbs[1], None))

    def use_native_callbacks(self, loss_addr, grad_addr, user):
        """C scorers given as raw function addresses (sr_loss_fn / sr_grad_fn) and their user pointer:
        a host port answering every scoring call without Python in the loop (bench's CPU baseline)."""
        self._cbs = (_lib.LOSS_FN(loss_addr), _lib.GRAD_FN(grad_addr) if grad_addr else _lib.GRAD_FN(), user)
        _lib.check(_lib.lib.sr_search_use_callbacks(self.h, self._cbs[0], self._cbs[1], user))

    def start(self, niterations):
        _lib.check(_lib.lib.sr_search_start(self.h, int(niterations)))

    def iterate(self):
        _lib.check(_lib.lib.sr_search_iterate(self.h))

    def head(self):
        _lib.check(_lib.lib.sr_search_head(self.h))

    def export(self) -> bytes:
        n = ctypes.c_int64()
        _lib.check(_lib.lib.sr_search_export(self.h, None, 0, ctypes.byref(n)))
        buf = ctypes.create_string_buffer(n.value)
        _lib.check(_lib.lib.sr_search_export(self.h, buf, n.value, ctypes.byref(n)))
        return buf.raw[: n.value]

    def import_(self, data: bytes):
        _lib.check(_lib.lib.sr_search_import(self.h, data, len(data)))

    def info(self) -> _lib.SrSearchInfo:
        inf = _lib.SrSearchInfo()
        _lib.check(_lib.lib.sr_search_get_info(self.h, ctypes.byref(inf)))
        return inf

    def members(self, which):
        """[PopMember] of island `which` (>= 0), the hall of fame (-1) or the Pareto front (-2)."""
        nm, nn = ctypes.c_int64(), ctypes.c_int64()
        _lib.check(_lib.lib.sr_search_member_count(self.h, int(which), ctypes.byref(nm), ctypes.byref(nn)))
        nm, nn = nm.value, nn.value
        offs = np.zeros(nm + 1, np.int64)
        deg, op, con = (np.zeros(max(nn, 1), np.uint8) for _ in range(3))
        feat = np.zeros(max(nn, 1), np.uint16)
        val = np.zeros(max(nn, 1), self.dtype)
        cost, loss = np.zeros(max(nm, 1), self.dtype), np.zeros(max(nm, 1), self.dtype)
        birth, ref, parent = (np.zeros(max(nm, 1), np.int64) for _ in range(3))
        comp = np.zeros(max(nm, 1), np.int32)
        p = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
        _lib.check(_lib.lib.sr_search_members(self.h, int(which), p(offs), p(deg), p(op), p(feat), p(con), p(val),
                                              p(cost), p(loss), p(birth), p(ref), p(parent), p(comp)))
        tb = TreeBatch(offs, deg[:nn], op[:nn], feat[:nn], con[:nn], val[:nn])
        return [PopMember(tb.tree(k), cost[k], loss[k], comp[k], parent[k], birth[k], ref[k]) for k in range(nm)]


def _torch_comm():
    """(rank, world, allgather_object) of the default torch.distributed group, or None."""
    try:
        import torch.distributed as tdist
    except ImportError:  # pragma: no cover
        return None
    if not (tdist.is_available() and tdist.is_initialized()) or tdist.get_world_size() == 1:
        return None
    if tdist.get_backend() != "gloo":
        # the exchange is a few KB of host objects; an "nccl" group would make torch initialise its
        # own HIP runtime on the GPU, which cannot share the device with the library's
        raise RuntimeError("equation_search(distributed=True) needs a gloo process group (CPU objects only)")
    world = tdist.get_world_size()

    def allgather(obj):
        out = [None] * world
        tdist.all_gather_object(out, obj)
        return out

    return tdist.get_rank(), world, allgather


def equation_search(X=None, y=None, *, niterations=10, options, weights=None, search_options=None, seed=0,
                    verbosity=0, dataset=None, distributed=False, scoring_lanes=4, _loss_fn=None, _grad_fn=None,
                    _native_scorer=None, _rank_share=None):
    """Batched-island ``equation_search`` (src/SymbolicRegression.jl:967-1216) -> SearchResult.

    distributed=True (torch.distributed initialised, one process per GPU; SURVEY §8(e) island
    sharding): island i lives on rank i % world; every rank scores only its islands' children (one
    batched launch per round on its own GPU); after each iteration the ranks all-gather their islands
    and every rank replays the head's island-by-island bookkeeping identically.
    scoring_lanes: device contexts (streams) the rank's islands are split over, one host thread each,
    so device round trips overlap; results do not depend on it (num_evals up to rounding).
    ``_loss_fn`` / ``_grad_fn`` replace the device scorer with CPU callbacks (tests only);
    ``_native_scorer`` (an object with ``loss_addr``, ``grad_addr``, ``user``: C callbacks) likewise,
    without Python in the loop (bench.py's CPU baseline).
    ``_rank_share=(r, N)`` (bench.py's island-sharding projection, one process): the engine of rank r
    of N — it advances only its own islands i % N == r and runs the head over all of them; the other
    ranks' islands are imported every iteration as they were initialised (helper engines started before
    the timed loop): the per-rank work of an N-rank search without the all-gather itself."""
    so = search_options or SearchOptions()
    comm = _torch_comm() if distributed else None
    rank, world, allgather = comm if comm else (0, 1, None)
    if _rank_share is not None:
        if comm:
            raise ValueError("_rank_share is a one-process measurement")
        rank, world = int(_rank_share[0]), int(_rank_share[1])
    if dataset is None:
        dataset = Dataset(np.asarray(X), np.asarray(y), weights=weights)
    def scorer(e, lanes):
        if _native_scorer is not None:
            e.use_native_callbacks(_native_scorer.loss_addr, _native_scorer.grad_addr, _native_scorer.user)
        elif _loss_fn is not None:
            e.use_callbacks(_loss_fn, _grad_fn)
        else:
            from .device import get_lane_context

            e.use_device(dataset)
            for lane in range(1, lanes):
                e.add_device(dataset, get_lane_context(lane))

    eng = NativeSearch(dataset, options, so, seed, rank, world)
    scorer(eng, max(1, min(int(scoring_lanes), len(range(rank, options.populations, world)))))
    stale = []
    if _rank_share is not None and world > 1:
        for r in range(world):
            if r != rank:
                h = NativeSearch(dataset, options, so, seed, r, world)
                scorer(h, 1)
                h.start(niterations)
                stale.append(h.export())
                del h
        allgather = lambda part: [part] + stale  # noqa: E731  (this rank's own part first: skipped below)
        rank_in_gather = 0
    else:
        rank_in_gather = rank

    def exchange():
        if world == 1 or allgather is None:
            return
        for r, part in enumerate(allgather(eng.export())):
            if r != rank_in_gather:
                eng.import_(part)

    t0 = time.perf_counter()
    eng.start(niterations)
    exchange()
    for it in range(niterations):
        eng.iterate()
        exchange()
        eng.head()
        if verbosity and rank == 0:
            front = eng.members(_lib.SR_SEARCH_PARETO)
            best = min(front, key=lambda m: m.loss)
            print(f"iteration {it + 1}/{niterations}: best loss {best.loss:.4g} (complexity {best.complexity})")
    exchange()  # the final migrations
    wall = time.perf_counter() - t0
    inf = eng.info()
    info = dict(num_evals=inf.num_evals, calls=inf.device_calls, dev=inf.device_ms, host=inf.host_ms,
                kernel=inf.kernel_ms)
    if world > 1 and allgather is not None and not stale:
        parts = allgather(info)
        info = {k: sum(p[k] for p in parts) for k in info}
    info_base = eng.info()
    dataset.use_baseline = bool(info_base.use_baseline)
    dataset.baseline_loss = dataset.dtype.type(info_base.baseline_loss)
    hof = HallOfFame(options.maxsize)
    for m in eng.members(_lib.SR_SEARCH_HALL_OF_FAME):
        hof.members[m.complexity - 1] = m
        hof.exists[m.complexity - 1] = True
    pops = [eng.members(i) for i in range(options.populations)]
    return SearchResult(hof, hof.pareto_frontier(), pops, niterations, wall, niterations * options.populations,
                        float(info["num_evals"]), int(info["calls"]), info["dev"] / 1e3, info["host"] / 1e3,
                        info["kernel"] / 1e3)
