#!/usr/bin/env python3
"""Benchmark: batched eval_loss throughput (BASELINE.json metric) on C2, with C4, tree sharding and the
search-iterations half of the metric as sub-objects.

One step = score the whole population once: compile the trees into device programs, upload, run
the interpreter over all rows, reduce, copy losses back, exact re-check when needed, finalize (the
full cost of one `eval_cost_batch` call of a search iteration).  Trees and data are synthetic
(seeded), generated before timing; the dataset is resident in HBM when the timed region starts.

  python bench.py [--gpus N] [--steps K] [--warmup W]

--gpus N without a launcher (WORLD_SIZE unset) starts N rank processes itself (fresh children of a
parent that makes no GPU call; rank 0 prints).  Under torch.distributed.run the launcher's ranks are
used.  One process per GPU (LOCAL_RANK); a gloo group is the CPU channel (unique id, barriers,
max-over-ranks timing); every data-path exchange is the library's own RCCL over xGMI.

Headline, C2 (BASELINE config 2): 10k trees x 1M rows x 5 features PER GPU, weak scaling.  N = 1:
  the single-GPU call (sr_eval_loss_batch).  N > 1: rank r holds its own 1M-row shard of an N x 1M-row
  dataset, and the step is the row-sharded call (sr_eval_loss_sharded: ONE RCCL all-reduce of packed
  per-tree partials).  `c2_sharded_path` (N = 1) times the same step through the row-sharded call at
  world size 1, so the scaling denominator's code path is on record.
Sub-objects measured at every N, each through the same code path at every N:
  c4            BASELINE config 4: 100k trees x 64M (2^26) rows, rows sharded n/N (strong scaling).
  tree_sharded  the C2 population over a replicated 1M-row dataset, trees dealt over the N ranks.
Rank 0 at N = 1 also reports: the interpreter roofline, the complete-trees-only and Float64 lines,
the CPU baseline (the C oracle on the host cores) and the parity of the timed step against it, and
the search throughput (C1 and C3) with the same engine scored by the C port as its CPU baseline.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "symbolicregression.jl_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

PEAK_FP32_TFLOPS = 157.3  # MI355X FP32 vector dense peak, MI355X_MICROARCH.md
PEAK_FP64_TFLOPS = 78.6   # MI355X FP64 vector dense peak
PEAK_HBM_GBPS = 8000.0
C2_OPS = dict(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp", "log"])
BLOCK = 1 << 20           # C4 data is generated in seeded 1M-row blocks (shards are whole blocks)


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=8)
    ap.add_argument("--rows", type=int, default=0, help="C2 rows per GPU (default 2^20)")
    ap.add_argument("--trees", type=int, default=0, help="C2 trees (default 10k)")
    ap.add_argument("--c4-rows", type=int, default=1 << 26, help="C4 total rows (multiple of 2^20 x N)")
    ap.add_argument("--c4-trees", type=int, default=100_000)
    ap.add_argument("--c4-steps", type=int, default=3)
    ap.add_argument("--no-c4", action="store_true")
    ap.add_argument("--no-c4-parity", action="store_true", help="skip the C4 full-size parity sample (N = 1)")
    ap.add_argument("--c4-parity-trees", type=int, default=64)
    ap.add_argument("--no-tree-sharded", action="store_true")
    ap.add_argument("--no-sharded-path", action="store_true", help="skip the N = 1 c2_sharded_path line")
    ap.add_argument("--cpu-trees", type=int, default=0, help="CPU-baseline tree sample (0 = auto, ~15 s)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extra", action="store_true", help="skip the complete-only and Float64 lines")
    ap.add_argument("--search-iters", type=int, default=40, help="iterations of the C1 / C3 searches (0 = skip)")
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher + CPU channel only (no device): rehearses --gpus N on a CPU host")
    ap.add_argument("--search-cpu-iters", type=int, default=0,
                    help="iterations of the CPU-port searches (0 = C1: all, C3: 2, a bounded sample)")
    return ap.parse_args(argv)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n):
    """`--gpus N` without a launcher: N fresh rank processes (this parent has made no GPU call and
    never re-execs); each inherits stdout, rank 0 prints the line.  A failed rank stops the others."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), SR_BENCH_SPAWNED="1")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    alive = set(range(n))
    while alive:
        for r in list(alive):
            code = procs[r].poll()
            if code is None:
                continue
            alive.discard(r)
            if code != 0:
                rc = rc or code
                for q in alive:
                    procs[q].terminate()
        time.sleep(0.05)
    return rc


def c2_data(n_rows, rank, nf=5, dtype=np.float32):
    rng = np.random.default_rng(2 + 1000 * rank)
    X = rng.standard_normal((nf, n_rows)).astype(dtype)
    y = (2 * np.cos(X[3]) + X[0] ** 2 - 2 + 0.1 * np.random.default_rng(3 + 1000 * rank).standard_normal(n_rows)
         ).astype(dtype)
    return X, y


def c4_shard(rank, world, rows_total, nf=5):
    """Rows [rank n/N, (rank+1) n/N) of the C4 dataset, built from seeded 1M-row blocks."""
    nblocks = rows_total // BLOCK
    b0, b1 = rank * nblocks // world, (rank + 1) * nblocks // world
    X = np.empty((nf, (b1 - b0) * BLOCK), dtype=np.float32)
    y = np.empty((b1 - b0) * BLOCK, dtype=np.float32)
    for j, b in enumerate(range(b0, b1)):
        rng = np.random.default_rng([4, b])
        xb = rng.standard_normal((nf, BLOCK), dtype=np.float32)
        X[:, j * BLOCK:(j + 1) * BLOCK] = xb
        y[j * BLOCK:(j + 1) * BLOCK] = 2 * np.cos(xb[3]) + xb[0] ** 2 - 2 + 0.1 * rng.standard_normal(BLOCK, dtype=np.float32)
    return X, y


class Comm:
    """The CPU channel: a gloo group (world 1 too, so the sharded code path is the same at every N)."""

    def __init__(self, world, rank):
        import torch.distributed as tdist

        self.d = tdist
        self.world, self.rank = world, rank
        addr = os.environ.get("MASTER_ADDR", "127.0.0.1")
        port = os.environ.get("MASTER_PORT") or str(_free_port())
        tdist.init_process_group("gloo", init_method=f"tcp://{addr}:{port}", rank=rank, world_size=world)

    def barrier(self):
        self.d.barrier()

    def max(self, v):
        import torch

        t = torch.tensor([float(v)], dtype=torch.float64)
        self.d.all_reduce(t, op=self.d.ReduceOp.MAX)
        return float(t.item())

    def close(self):
        self.d.destroy_process_group()


def progress(msg):
    """A progress line on stderr (long runs: the bench's phases each print one as they start)."""
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def timed(step, steps, warmup, barrier):
    """W untimed steps, then K timed steps between barriers (every library call returns after its
    streams have drained: the device is synchronised on both sides)."""
    for _ in range(warmup):
        step()
    barrier()
    kernel_ms, stamps = [], []
    t0 = time.perf_counter()
    for _ in range(steps):
        kernel_ms.append(step())
        stamps.append(time.perf_counter())
    barrier()
    dt = time.perf_counter() - t0
    step_ms = np.diff(np.array([t0] + stamps)) * 1e3
    return dt, step_ms, kernel_ms


def lib_step(ctx, fn, state):
    """Wrap one library call: its interpreter kernel time (sum of launches), busy time (union) and launches."""
    def step():
        fn()
        k, _ = ctx.last_kernel_ms()
        state.setdefault("busy", []).append(ctx.last_busy_ms())
        state.setdefault("launches", []).append(ctx.last_launches())
        return k
    return step


def single_gpu_call(ctx, tb, ds, opts, dtype=np.float32):
    import ctypes

    from sr_amd import _lib

    dsh = ds.device_handle(ctx)
    oid = ctx.opset_id(opts.operators)
    s = tb.to_struct()
    out = {"loss": np.empty(tb.n_trees, dtype=dtype), "comp": np.empty(tb.n_trees, dtype=np.uint8)}

    def call():
        _lib.check(_lib.lib.sr_eval_loss_batch(ctx.handle, dsh, oid, ctypes.byref(s), None, 0, 0,
                                               out["loss"].ctypes.data_as(ctypes.c_void_p),
                                               out["comp"].ctypes.data_as(ctypes.c_void_p)))
    return call, out


def roofline(flops, kernel_ms, peak, **extra):
    achieved = flops / (kernel_ms * 1e-3) / 1e12
    out = {"bound": "valu", "achieved": achieved, "peak": peak, "unit": "TFLOP/s", "frac": achieved / peak,
           "kernel_ms_per_step": kernel_ms, "flops_per_step": flops}
    out.update(extra)
    return out


def main():
    args = parse_args()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))

    if args.dry_run:
        comm = Comm(world, rank)
        dt, step_ms, _ = timed(lambda: time.sleep(0.001 * (1 + rank)), args.steps, args.warmup, comm.barrier)
        dt = comm.max(dt)
        if rank == 0:
            print(json.dumps({"dry_run": True, "n_gpus": world, "steps": args.steps, "ms_per_step": dt / args.steps * 1e3,
                              "ranks_launched_by": "bench.py" if os.environ.get("SR_BENCH_SPAWNED") else "launcher"}),
                  flush=True)
        comm.close()
        return

    import sr_amd  # noqa: E402  (after the spawn decision: the parent never loads the HIP runtime)
    from sr_amd import Dataset, Options, flatten_trees, gen_random_batch, gen_random_population
    from sr_amd.distributed import comm_info, eval_loss_sharded, eval_loss_tree_sharded, init_device_comm

    comm = Comm(world, rank)
    # the device: LOCAL_RANK, or SR_AMD_DEVICE (a rehearsal on a one-GPU box puts every rank on device 0;
    # RCCL refuses two ranks on one device, so that run takes the gloo exchange below)
    ctx = sr_amd.get_context(int(os.environ.get("SR_AMD_DEVICE", local_rank)))
    # the library's RCCL communicator (every data-path exchange of the sharded calls); if it cannot be
    # created on every rank, all ranks fall back to the library's host transport (the same C++ sharded
    # path, its collectives staged through host memory over gloo) and the line says so, rather than
    # printing nothing
    err = None
    try:
        init_device_comm(ctx=ctx)
    except Exception as e:  # noqa: BLE001  (reported in the JSON line)
        if world == 1:
            raise
        err = f"{type(e).__name__}: {e}"
    if world > 1 and comm.max(1.0 if err else 0.0) > 0.0:
        if ctx.has_comm:
            from sr_amd.distributed import destroy_device_comm
            destroy_device_comm(ctx)
        print(f"[bench] rank {rank}: RCCL communicator unavailable ({err or 'failed on a peer rank'}); "
              "the sharded calls exchange over gloo (host transport)", file=sys.stderr, flush=True)
        from sr_amd.distributed import init_host_comm
        init_host_comm(ctx=ctx)
        cinfo = {"nranks": None, "rccl_error": err or "failed on a peer rank", "transport": "host (gloo)"}
    else:
        cinfo = comm_info(ctx)

    opts = Options(**C2_OPS)
    nt = args.trees or 10_000
    trees = gen_random_population(nt, opts, 5, max_size=30, seed=1)
    tb = flatten_trees(trees, np.float32)
    rows = args.rows or (1 << 20)
    rows_total = rows * world
    X, y = c2_data(rows, rank)
    ds = Dataset(X, y)
    ds.device_handle(ctx)  # upload before timing
    nodes, ops = int(tb.n_nodes), int(tb.n_operator_nodes)

    # ---- headline: C2, weak scaling
    if rank == 0:
        progress(f"C2 headline: {nt} trees x {rows} rows, {args.warmup} + {args.steps} steps")
    state = {}
    if world == 1:
        call, out = single_gpu_call(ctx, tb, ds, opts)
        path = "single-GPU sr_eval_loss_batch"
    else:
        out = {}

        def call():
            out["loss"], out["comp"] = eval_loss_sharded(tb, ds, opts)
        path = "row-sharded sr_eval_loss_sharded (one RCCL all-reduce of packed [5, n_trees] partials per step)"
    dt, step_ms, kernel_ms = timed(lib_step(ctx, call, state), args.steps, args.warmup, comm.barrier)
    dt = comm.max(dt)
    comp = np.asarray(out["comp"]).astype(bool)
    loss = np.asarray(out["loss"]).copy()
    value = float(nodes) * float(rows_total) * args.steps / dt
    kmean = float(np.mean(kernel_ms))
    busy = float(np.mean(state["busy"][-args.steps:]))
    n_launch = int(round(float(np.mean(state["launches"][-args.steps:]))))
    flops_per_step = float(rows) * (ops + 3 * nt)  # this GPU's interpreter work per step
    traffic = measured_traffic("c2", nt, rows)
    rpl = ctx.last_rows_per_lane()
    n_derived = ctx.last_derived_columns()
    n_exact_last, n_fold_last = ctx.last_exact_trees(), ctx.last_fold_trees()
    ref_fold = ctx.last_ref_fold()

    subs = {}
    if world == 1:  # the fold's cost on the headline step: the same step with the f64 sums
        ctx.set_tuning("ref_fold", 0)
        call0, _ = single_gpu_call(ctx, tb, ds, opts)
        st0 = {}
        dt0, _, km0 = timed(lib_step(ctx, call0, st0), max(3, args.steps // 2), 2, comm.barrier)
        ctx.set_tuning("ref_fold", 1)
        subs["fold_cost"] = {
            "ms_per_step_fold": dt / args.steps * 1e3, "ms_per_step_f64_sum": dt0 / max(3, args.steps // 2) * 1e3,
            "fold_kernel_ms_per_step": ref_fold["kernel_ms"], "trees_folded": ref_fold["folded"],
            "trees_fallback": ref_fold["fallback"], "path": ref_fold["path"],
            "note": ("ref_fold 1 (default): every complete tree's loss is the reference's in-order Float32 fold; "
                     "ref_fold 0: the f64 per-tree sums of rounds 1-5 (~5e-4 relative off at 2^20 rows)")}
    if world == 1 and not args.no_sharded_path:
        if rank == 0:
            progress("c2_sharded_path")
        subs["c2_sharded_path"] = sharded_path_line(ctx, tb, ds, opts, eval_loss_sharded, args, comm, nodes, rows)
    if not args.no_tree_sharded:
        if rank == 0:
            progress("tree_sharded")
        subs["tree_sharded"] = tree_sharded_line(ctx, tb, opts, eval_loss_tree_sharded, args, comm, world, rank,
                                                 nodes, rows, loss if world == 1 else None, comp if world == 1 else None)
    if not args.no_c4:
        if rank == 0:
            progress("c4")
        subs["c4"] = c4_line(ctx, opts, eval_loss_sharded, gen_random_batch, Dataset, args, comm, world, rank)

    extra = {}
    if rank == 0 and world == 1 and not args.no_extra:
        progress("complete-only and Float64 lines")
        extra = extra_lines(ctx, opts, trees, comp, X, y, args)
    cpu, parity = None, None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        progress("CPU baseline and parity")
        cpu, parity = cpu_baseline_and_parity(opts, tb, X, y, args.cpu_trees, loss, comp)
    search = None
    if rank == 0 and world == 1 and args.search_iters > 0:
        search = search_lines(args)

    if rank == 0:
        algo_bytes = algorithmic_bytes(nt, rows, n_launch, rpl)
        algo_bytes_d = algorithmic_bytes(nt, rows, n_launch, rpl, n_derived)
        line = {
            "metric": "tree-node x row evals/sec (batched eval_loss, fp32)",
            "value": value,
            "unit": "node-evals/s",
            "n_gpus": world,
            "world_size_rccl": cinfo["nranks"],
            **({"rccl_error": cinfo["rccl_error"], "transport": cinfo["transport"]} if cinfo.get("rccl_error") else {}),
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": dt / args.steps * 1e3,
            "step_ms_min_median_max": [float(step_ms.min()), float(np.median(step_ms)), float(step_ms.max())],
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (seeded): gen_random_tree_fixed_size population, X~N(0,1), y=2cos(x4)+x1^2-2+0.1N",
            "config": {
                "workload": (f"C2 batched eval_loss: {nt // 1000}k random trees (size U{{1..30}}; +,-,*,/,cos,exp,"
                             f"safe_log) x {rows >> 20}M rows x 5 features per GPU"),
                "n_trees": nt,
                "tree_nodes": nodes,
                "operator_nodes": ops,
                "rows_per_gpu": rows,
                "rows_total": rows_total,
                "nfeatures": 5,
                "parallelism": (f"rows sharded x{world}; one RCCL all-reduce of packed [5, n_trees] per-tree partials"
                                if world > 1 else "single GPU"),
                "code_path": path,
                "fraction_complete": float(np.mean(comp)),
                "exact_trees": n_exact_last,
                "fold_trees": n_fold_last,
                "loss_accumulation": ("every complete tree's loss is the reference's in-order fold in Float32 "
                                      "(LossFunctions.jl:38-58), bit for bit given the element losses; inside the "
                                      "timed step (DESIGN §4.4)" if ref_fold["path"] > 0 or world > 1 else
                                      "f64 per-tree sums (ref_fold off)"),
                "ref_fold": ref_fold,
                "runtime": {"hip": cinfo.get("hip"), "rccl": cinfo.get("rccl")},
            },
            "roofline": roofline(
                flops_per_step, kmean, PEAK_FP32_TFLOPS,
                busy_ms_per_step=busy,
                traffic=traffic.get("hbm_read_bytes_per_step") if traffic else None,
                traffic_source=traffic.get("source") if traffic else None,
                kernel=(f"sr_tile_kernel<float,{rpl},LOSS,gather=false,BASIC,W=4,L2"
                        + (",register stack>" if rpl >= 16 else ">")),
                launches_per_step=n_launch,
                kernel_ms_convention=("per step: sum of the interpreter launches' HIP-event durations on the "
                                      "library's streams (= the kernel-trace sum); busy_ms_per_step = the union "
                                      "of those intervals (the two pipeline streams overlap)"),
                flop_convention="n_rows * sum_t(n_op(t) + 3), 1 flop per operator incl. transcendentals (SURVEY 8d)",
                algorithmic_bytes_per_step=algo_bytes,
                algorithmic_GBps=algo_bytes / (kmean * 1e-3) / 1e9,
                algorithmic_bytes_with_derived_per_step=algo_bytes_d,
                n_derived_columns=n_derived,
                bytes_convention=("ceil(n_trees/G) passes x (nf+1) x n_rows x 4 B; X/y re-reads are served from "
                                  "L2/MALL; _with_derived adds the derived columns (n_derived x n_rows x 4 B per pass)"),
            ),
            "cpu_baseline": cpu,
            "parity": parity,
            "search": search,
        }
        line.update(subs)
        line.update(extra)
        print(json.dumps(compact_line(line)), flush=True)
    comm.close()


# keys of the printed line's sub-objects kept inline; everything else (held-tree expressions, per-bucket
# gradient tables, projection internals, phase breakdowns) goes to the detail file only.  Round 5's
# 20.9 KB line was not parsed by the driver: the printed line stays well under 12 KB.
_KEEP = {
    "roofline": ("bound", "achieved", "peak", "unit", "frac", "traffic", "kernel_ms_per_step", "busy_ms_per_step",
                 "flops_per_step", "kernel", "algorithmic_bytes_per_step", "algorithmic_GBps", "launches_per_step",
                 "n_trees", "ms_per_step", "node_evals_per_s", "hbm_GBps", "kernel_sum_ms_per_step",
                 "fraction_complete"),
    "parity": ("trees", "rows", "complete", "flags_bit_exact", "flag_mismatches", "max_rel_vs_f64_accum",
               "median_rel_vs_f64_accum", "n_held_to_libm_spread_bar", "loss_failures_vs_f64_accum",
               "max_rel_vs_ref_f32_fold", "median_rel_vs_ref_f32_fold", "n_bit_exact_vs_ref_f32_fold",
               "loss_failures_vs_ref_fold", "ref_fold_inf_trees", "ref_fold_inf_mismatches", "accumulation", "pass",
               "max_rel", "median_rel", "loss_failures", "cpu_s"),
}


def _pick(d, keys):
    return {k: d[k] for k in keys if isinstance(d, dict) and k in d}


def compact_line(line):
    """The printed JSON line: the contract's keys and each sub-object's headline numbers.  The full line
    (every held tree, gradient bucket and projection input) is written to the detail file
    (SR_BENCH_DETAIL, default gpurun_out/bench_detail.json) and named in the line."""
    path = os.environ.get("SR_BENCH_DETAIL", os.path.join(ROOT, "gpurun_out", "bench_detail.json"))
    try:
        os.makedirs(os.path.dirname(path), exist_ok=True)
        with open(path, "w") as f:
            json.dump(line, f)
    except OSError:
        path = None
    out = {k: v for k, v in line.items()
           if k not in ("roofline", "parity", "search", "c4", "tree_sharded", "c2_sharded_path", "f64",
                        "roofline_complete_only", "config")}
    cfg = dict(line.get("config") or {})
    out["config"] = cfg
    out["roofline"] = _pick(line.get("roofline") or {}, _KEEP["roofline"])
    par = line.get("parity")
    out["parity"] = _pick(par, _KEEP["parity"]) if par else par
    if "roofline_complete_only" in line:
        out["roofline_complete_only"] = _pick(line["roofline_complete_only"], _KEEP["roofline"])
    if "f64" in line:
        f = line["f64"]
        out["f64"] = dict(_pick(f, _KEEP["roofline"]), parity=_pick(f.get("parity") or {}, _KEEP["parity"]))
    if "c2_sharded_path" in line:
        out["c2_sharded_path"] = _pick(line["c2_sharded_path"], ("ms_per_step", "value", "kernel_ms_per_step"))
    if "tree_sharded" in line:
        t = line["tree_sharded"]
        out["tree_sharded"] = _pick(t, ("value", "unit", "ms_per_step", "scaling", "n_gpus", "equals_single_gpu",
                                        "single_call_ms_per_step", "overhead_vs_single_call"))
        for k in ("projection_8_ranks", "projection_8_ranks_100k_trees"):
            if k in t:
                out["tree_sharded"][k] = _pick(t[k], ("rank0_share_ms", "single_call_ms", "efficiency_excluding_allgather"))
    if "c4" in line:
        c = line["c4"]
        o = _pick(c, ("value", "unit", "ms_per_step", "steps", "n_gpus", "scaling", "rows_per_gpu", "n_trees",
                      "fraction_complete", "skipped", "loss_accumulation"))
        if "roofline" in c:
            o["roofline"] = _pick(c["roofline"], _KEEP["roofline"])
        lp = c.get("last_step_passes") or {}
        o["passes"] = _pick(lp, ("exact_trees", "fold_trees", "ref_fold_trees", "fold_segments_row_by_row"))
        if "projection_8_ranks" in c:
            o["projection_8_ranks"] = _pick(c["projection_8_ranks"], ("projected_ms_per_step", "efficiency"))
        if "parity" in c:
            p = c["parity"]
            o["parity"] = {"pass": p.get("pass"), "rows": p.get("rows"), "accumulation": p.get("accumulation")}
            for k in ("sample", "planted_big"):
                if k in p:
                    o["parity"][k] = _pick(p[k], ("trees", "complete", "flag_mismatches", "ref_fold_inf_mismatches",
                                                  "max_rel_vs_f64_accum", "max_rel_vs_ref_f32_fold",
                                                  "max_rel_device_vs_ref_f32_fold",
                                                  "n_held_to_libm_spread_bar", "loss_failures",
                                                  "n_bit_exact_vs_ref_f32_fold"))
        out["c4"] = o
    if line.get("search"):
        s = {}
        for name, v in line["search"].items():
            o = _pick(v, ("value", "unit", "iterations_per_s", "iterations_per_s_f64_sum",
                          "device_wall_per_call_us_f64_sum", "islands", "wall_s", "device_calls",
                          "device_wall_per_call_us", "kernel_busy_per_call_us", "best_loss"))
            if "cpu_baseline" in v:
                o["cpu_baseline"] = _pick(v["cpu_baseline"], ("value", "unit", "iterations_per_s", "cores", "kind"))
            if "grad_roofline" in v:
                o["grad_roofline"] = _pick(v["grad_roofline"], ("achieved", "peak", "unit", "frac", "kernel_ms_per_call"))
            if "projection_8_ranks" in v:
                pr = v["projection_8_ranks"]
                o["projection_8_ranks"] = dict(_pick(pr, ("speedup", "efficiency")),
                                               weak_efficiency=(pr.get("weak_scaling") or {}).get("efficiency"))
            s[name] = o
        out["search"] = s
    out["detail_file"] = os.path.relpath(path, ROOT) if path else None
    return out


def sharded_path_line(ctx, tb, ds, opts, eval_loss_sharded, args, comm, nodes, rows):
    """The C2 step through the row-sharded call at world size 1 (the code path every N > 1 runs)."""
    st = {}
    res = {}

    def call():
        res["l"], res["c"] = eval_loss_sharded(tb, ds, opts)
    dt, step_ms, kms = timed(lib_step(ctx, call, st), args.steps, args.warmup, comm.barrier)
    return {"ms_per_step": dt / args.steps * 1e3, "value": float(nodes) * rows * args.steps / dt,
            "kernel_ms_per_step": float(np.mean(kms)), "busy_ms_per_step": float(np.mean(st["busy"][-args.steps:])),
            "derived_columns": ctx.last_derived_columns(), "exact_trees": ctx.last_exact_trees(),
            "what": "C2 through sr_eval_loss_sharded at world size 1 (the N > 1 code path)"}


def tree_sharded_line(ctx, tb, opts, eval_loss_tree_sharded, args, comm, world, rank, nodes, rows, ref_loss, ref_comp):
    """The C2 population over one replicated 1M-row dataset (rank 0's data on every rank), trees dealt
    over the ranks: strong scaling of tree sharding."""
    from sr_amd import Dataset

    X, y = c2_data(rows, 0)
    ds = Dataset(X, y)
    ds.device_handle(ctx)
    res = {}

    def step():
        t = time.perf_counter()
        res["l"], res["c"] = eval_loss_tree_sharded(tb, ds, opts)
        return (time.perf_counter() - t) * 1e3
    steps, warm = max(5, args.steps // 2), 3
    dt, step_ms, _ = timed(step, steps, warm, comm.barrier)
    dt = comm.max(dt)
    out = {"value": float(nodes) * rows * steps / dt, "unit": "node-evals/s", "ms_per_step": dt / steps * 1e3,
           "scaling": "strong", "n_gpus": world,
           "workload": f"C2 population ({tb.n_trees} trees) x {rows >> 20}M rows replicated, trees dealt over {world} ranks"}
    if ref_comp is not None:  # N = 1: the same answer as the single-GPU call
        out["equals_single_gpu"] = bool(np.array_equal(res["c"], ref_comp) and
                                        np.array_equal(res["l"][ref_comp], ref_loss[ref_comp]))
    if world == 1:
        # the overhead of the tree-sharded call at world 1 (<= 1.05x the single call on the
        # same dataset), and the 8-rank projection: rank 0's share under the owners rule, scored by the
        # single-GPU call (the per-rank work at N = 8; the results all-gather is not included)
        from sr_amd.distributed import tree_owners

        call, _ = single_gpu_call(ctx, tb, ds, opts)

        def single():
            t = time.perf_counter()
            call()
            return (time.perf_counter() - t) * 1e3
        dt1, _, _ = timed(single, steps, warm, comm.barrier)
        share = tb.take(np.nonzero(tree_owners(tb, 8) == 0)[0])
        call8, _ = single_gpu_call(ctx, share, ds, opts)

        def single8():
            t = time.perf_counter()
            call8()
            return (time.perf_counter() - t) * 1e3
        dt8, _, _ = timed(single8, steps, warm, comm.barrier)
        t1, t8 = dt1 / steps * 1e3, dt8 / steps * 1e3
        out["single_call_ms_per_step"] = t1
        out["overhead_vs_single_call"] = out["ms_per_step"] / t1
        out["projection_8_ranks"] = {"rank0_share_trees": share.n_trees, "rank0_share_ms": t8,
                                     "efficiency_excluding_allgather": t1 / (8 * t8)}
        # tree sharding's own regime: a population ten times C2's (100k trees, the C4 generator) over the
        # same replicated 1M rows — the per-call fixed costs (compile of the first chunk, exact pass,
        # launch latency) amortise over 12.5k trees per rank
        from sr_amd import gen_random_batch

        big = gen_random_batch(100_000, opts, 5, max_size=30, seed=4)
        callb, _ = single_gpu_call(ctx, big, ds, opts)
        share_b = big.take(np.nonzero(tree_owners(big, 8) == 0)[0])
        callb8, _ = single_gpu_call(ctx, share_b, ds, opts)

        def run(c):
            def f():
                t = time.perf_counter()
                c()
                return (time.perf_counter() - t) * 1e3
            return f
        dtb, _, _ = timed(run(callb), 5, 2, comm.barrier)
        dtb8, _, _ = timed(run(callb8), 5, 2, comm.barrier)
        tb1, tb8 = dtb / 5 * 1e3, dtb8 / 5 * 1e3
        out["projection_8_ranks_100k_trees"] = {"trees": int(big.n_trees), "single_call_ms": tb1,
                                                "rank0_share_trees": int(share_b.n_trees), "rank0_share_ms": tb8,
                                                "efficiency_excluding_allgather": tb1 / (8 * tb8)}
    ds.free_device()
    return out


def c4_line(ctx, opts, eval_loss_sharded, gen_random_batch, Dataset, args, comm, world, rank):
    """BASELINE config 4: 100k trees x 64M rows sharded n/N, through sr_eval_loss_sharded at every N."""
    rows_total = args.c4_rows
    if rows_total % (BLOCK * world):
        return {"skipped": f"C4 total rows {rows_total} is not a multiple of 2^20 x {world}"}
    tb = gen_random_batch(args.c4_trees, opts, 5, max_size=30, seed=4)
    X, y = c4_shard(rank, world, rows_total)
    ds = Dataset(X, y)
    ds.device_handle(ctx)
    del X, y
    st = {}
    res = {}

    def call():
        res["l"], res["c"] = eval_loss_sharded(tb, ds, opts)
    if rank == 0:
        progress(f"c4 steps: {tb.n_trees} trees x {rows_total} rows / {world}")
    dt, step_ms, kms = timed(lib_step(ctx, call, st), args.c4_steps, 1, comm.barrier)
    dt = comm.max(dt)
    c4_fold = ctx.last_ref_fold()  # (2^26 rows: past fold_rows_max, the f64 sums)
    n_local = rows_total // world
    kmean, busy = float(np.mean(kms)), float(np.mean(st["busy"][-args.c4_steps:]))
    flops = float(n_local) * (tb.n_operator_nodes + 3 * tb.n_trees)
    traffic = measured_traffic("c4", tb.n_trees, n_local)
    nl = int(round(float(np.mean(st["launches"][-args.c4_steps:]))))
    algo = algorithmic_bytes(tb.n_trees, n_local, nl, ctx.last_rows_per_lane())
    n_derived = ctx.last_derived_columns()
    algo_d = algorithmic_bytes(tb.n_trees, n_local, nl, ctx.last_rows_per_lane(), n_derived)
    fi = ctx.last_fold_info()
    passes = {"exact_trees": ctx.last_exact_trees(), "fold_trees": ctx.last_fold_trees(),
              "phase_ms": [round(float(v), 3) for v in ctx.last_phase_ms()],
              "exact_kernel_ms": round(ctx.last_exact_kernel_ms(), 3),
              "fold_device_ms": {k: round(v, 3) for k, v in ctx.last_fold_ms().items()},
              "fold_segments_row_by_row": fi[1], "fold_segment_rows": fi[2]}
    out = {"metric": "tree-node x row evals/sec (batched eval_loss, fp32)",
           "value": float(tb.n_nodes) * rows_total * args.c4_steps / dt, "unit": "node-evals/s",
           "ms_per_step": dt / args.c4_steps * 1e3, "steps": args.c4_steps, "warmup": 1, "n_gpus": world,
           "scaling": "strong",
           "workload": (f"C4 row-sharded eval_loss: {tb.n_trees // 1000}k random trees (size U{{1..30}}; native "
                        f"generator, seed 4) x {rows_total >> 20}M rows x 5 features, rows sharded n/{world}"),
           "code_path": "sr_eval_loss_sharded (same at every N)", "rows_per_gpu": n_local, "n_trees": int(tb.n_trees),
           "fraction_complete": float(np.mean(res["c"])),
           "last_step_passes": dict(passes, note=("trees through the exact isfinite(sum) pass (BIG) and through the "
                                                   "in-order loss fold (sr_fold.h); phase_ms = sr_last_phase_ms")),
           "roofline": roofline(flops, kmean, PEAK_FP32_TFLOPS, busy_ms_per_step=busy, launches_per_step=nl,
                                kernel=f"sr_tile_kernel<float,{ctx.last_rows_per_lane()},LOSS,gather=false,BASIC,W=4,L2>",
                                algorithmic_bytes_per_step=algo, algorithmic_GBps=algo / (kmean * 1e-3) / 1e9,
                                algorithmic_bytes_with_derived_per_step=algo_d, n_derived_columns=n_derived,
                                traffic=traffic.get("hbm_read_bytes_per_step") if traffic else None,
                                traffic_source=traffic.get("source") if traffic else None,
                                hbm_GBps=(traffic["hbm_read_bytes_per_step"] / (kmean * 1e-3) / 1e9
                                          if traffic else None), hbm_peak_GBps=PEAK_HBM_GBPS)}
    if world == 1 and rank == 0:
        progress("c4 projection to 8 ranks (rank 0's 8M-row shard)")
        # (rank 0 of the 8-rank run folds as the whole 2^26-row call does: here, not at all)
        ctx.set_tuning("ref_fold", 1 if c4_fold["path"] > 0 else 0)
        out["projection_8_ranks"] = c4_projection(ctx, opts, tb, eval_loss_sharded, Dataset, args, comm, rows_total,
                                                  out["ms_per_step"], passes)
        ctx.set_tuning("ref_fold", 1)
    if world == 1 and rank == 0 and not args.no_c4_parity:
        progress("c4 parity (oracle over all rows for a tree sample)")
        # (2^26 rows: past fold_rows_max the f64 sums, ref_fold path 0)
        folded = c4_fold["path"] > 0
        out["loss_accumulation"] = ("the reference's in-order fold in Float32" if folded else
                                    "f64 per-tree sums: 2^26 rows pass fold_rows_max (2^24), where the reference's "
                                    "Float32 fold stalls up to 50 % below the exact mean (DESIGN 4.4)")
        out["parity"] = c4_parity(opts, tb, res, lambda t: eval_loss_sharded(t, ds, opts), rows_total,
                                  args.c4_parity_trees, accum="ref" if folded else "f64")
    ds.free_device()
    return out


# latency of one small collective (an error-word agreement, a gather of a few KB) and of the packed
# [5, 100k] f64 all-reduce over xGMI at 8 ranks, as assumed by the projection (not measured here: the
# driver's 8-GPU run is the first multi-rank one)
COLL_SMALL_MS, COLL_PACKED_MS = 0.05, 0.2


def c4_projection(ctx, opts, tb, eval_loss_sharded, Dataset, args, comm, rows_total, t1_ms, passes):
    """C4 at 8 ranks, projected from one GPU: rank 0's shard (rows [0, n/8)) through
    the same sharded call at world size 1 — compile, probe, interpreter and exact pass over its 8M rows —
    plus the terms the single shard does not see: the in-order loss fold's parallel phases (PRED pass,
    segment sums, composed steps) at 1/8 of the 1-GPU step's, its chain in full (the shards run it one
    after another), and the collectives (the packed all-reduce and ~14 small ones, assumed latencies)."""
    X, y = c4_shard(0, 8, rows_total)
    ds = Dataset(X, y)
    ds.device_handle(ctx)
    del X, y
    st = {}

    def call():
        eval_loss_sharded(tb, ds, opts)
    steps = max(2, args.c4_steps)
    dt, step_ms, _ = timed(lib_step(ctx, call, st), steps, 1, comm.barrier)
    shard_ms = dt / steps * 1e3
    shard_phases = [round(float(v), 3) for v in ctx.last_phase_ms()]
    ds.free_device()
    f = passes.get("fold_device_ms", {})
    fold_par = (f.get("pred", 0.0) + f.get("segsum", 0.0) + f.get("segtab", 0.0)) / 8.0
    fold_chain = f.get("chain", 0.0)
    n_small = 14 if passes.get("fold_trees", 0) else 4
    coll = COLL_PACKED_MS + n_small * COLL_SMALL_MS
    t8 = shard_ms + fold_par + fold_chain + coll
    return {"rank0_shard_rows": rows_total // 8, "rank0_shard_ms_per_step": shard_ms,
            "rank0_shard_phase_ms": shard_phases, "fold_parallel_ms_over_8": fold_par, "fold_chain_ms": fold_chain,
            "collectives_ms_assumed": coll, "projected_ms_per_step": t8, "one_gpu_ms_per_step": t1_ms,
            "efficiency": t1_ms / (8.0 * t8),
            "model": ("t8 = rank 0's 8M-row shard through sr_eval_loss_sharded at world 1 (measured) + the 1-GPU "
                      "step's fold PRED / segment-sum / composed-step device time / 8 + its fold chain (sequential "
                      f"over the shards) + collectives ({COLL_PACKED_MS} ms packed all-reduce + {n_small} x "
                      f"{COLL_SMALL_MS} ms small ones, assumed); efficiency = t1 / (8 t8)")}


_LIBM_EXACT_UNARY = {"neg", "square", "cube", "abs", "sign", "relu", "inv", "round", "floor", "ceil", "sqrt",
                     "safe_sqrt"}


def held_trees(opts, orc, sub, X, y, rows, d_loss, l64, bar, threads, ids=None, limit=40, accum="ref"):
    """For every tree held to its libm-spread bar (device vs the oracle past the plain relative bar;
    accum: the oracle's loss accumulation, the reference's in-order fold by default): the expression,
    the relative difference, and the operator whose +-1-ulp last-bit
    differences the tree's loss amplifies most — the oracle's conditioning probe restricted to one
    operator at a time (oracle/de_eval_impl.h perturb codes), four sign patterns each."""
    from sr_amd.node import string_tree

    out = []
    ops = opts.operators
    for j, k in enumerate(rows[:limit]):
        progress(f"held tree {j + 1} of {min(len(rows), limit)}")
        one = sub.take([k])
        present = set()
        for d, o in zip(one.degree, one.op):
            if d == 1 and ops.unaops[o - 1] not in _LIBM_EXACT_UNARY:
                present.add((ops.unaops[o - 1], 1))
            elif d == 2 and ops.binops[o - 1] in ("^", "safe_pow", "pow"):
                present.add((ops.binops[o - 1], 2))
        l0, _ = orc.eval_loss_batch(one, X, y, accum=accum, n_threads=threads)
        spreads = {}
        for name, deg in sorted(present):
            s = 0.0
            for seed in (1, 2, 3, 4):
                lp, cp = orc.eval_loss_batch(one, X, y, accum=accum, n_threads=threads,
                                             perturb=seed | orc.perturb_code(name, deg))
                dd = abs(float(lp[0]) - float(l0[0]))
                if cp[0] and np.isfinite(dd):
                    s = max(s, dd)
            spreads[name] = s / max(abs(float(l0[0])), 1e-300)
        amp = max(spreads, key=spreads.get) if spreads else None
        ref = float(l64[k])
        out.append({"tree": int(ids[k] if ids is not None else k), "expr": string_tree(sub.tree(int(k)), ops),
                    "rel": abs(float(d_loss[k]) - ref) / max(abs(ref), 1e-300),
                    "bar_rel": float(bar[k]) / max(abs(ref), 1e-300),
                    "amplified_op": amp, "rel_spread_per_op": spreads})
    return out


def per_tree_bar(orc, sub, X, y, d_loss, l64, ok, rel_bar, threads, accum="ref"):
    """The tests' per-tree loss bar (tests/parity_util.py): max(rel_bar |oracle|, 4 x the tree's spread
    under +-1-ulp libm perturbations), the spread measured only for the trees the plain bar misses
    (l64: the oracle's losses under accum)."""
    with np.errstate(invalid="ignore", divide="ignore"):
        r = np.where(d_loss == l64, 0.0, np.abs(d_loss - l64) / np.maximum(np.abs(l64), 1e-300))
    worst = np.nonzero(ok & (r > rel_bar))[0]
    spread = np.zeros(len(d_loss))
    if worst.size:
        progress(f"per-tree libm spread of {worst.size} trees")
        wsub = sub.take(worst)
        l0, c0 = orc.eval_loss_batch(wsub, X, y, accum=accum, n_threads=threads)
        for seed in (1, 2, 3, 4):
            lp, cp = orc.eval_loss_batch(wsub, X, y, accum=accum, n_threads=threads, perturb=seed)
            with np.errstate(invalid="ignore"):
                d = np.abs(lp.astype(np.float64) - l0.astype(np.float64))
            spread[worst] = np.maximum(spread[worst], np.where(cp & c0 & np.isfinite(d), d, 0.0))
    with np.errstate(invalid="ignore"):
        bar = np.maximum(rel_bar * np.abs(l64), 4 * spread)
        err = np.where(d_loss == l64, 0.0, np.abs(d_loss - l64))
    return r, bar, err, int(worst.size)


def c4_parity(opts, tb, res, device_call, rows_total, n_sample, accum="ref"):
    """C4 at full size against the oracle: a stratified sample of the timed step's trees (complete and
    incomplete, every size) over all rows, plus planted trees whose values reach the exact-sum
    threshold (max|v| >= floatmax / 2n: DynamicExpressions' isfinite(sum) decided in Julia's pairwise
    order over 2^26 rows, BIG path) scored by the same sharded call; flags bit-exact, +Inf exactly where
    the reference's Float32 fold is +Inf, losses within the per-tree bar."""
    from oracle import Oracle
    from sr_amd import flatten_trees, parse_expression

    threads = min(int(os.environ.get("OMP_NUM_THREADS", "0")) or (os.cpu_count() or 1), 16)
    t0 = time.perf_counter()
    comp = np.asarray(res["c"]).astype(bool)
    sizes = np.diff(np.asarray(tb.offsets))
    pick = []
    for want_comp, k in ((True, n_sample * 3 // 4), (False, n_sample - n_sample * 3 // 4)):
        cand = np.nonzero(comp == want_comp)[0]
        cand = cand[np.argsort(sizes[cand], kind="stable")]  # every size: evenly over the size order
        pick.extend(cand[np.linspace(0, len(cand) - 1, k).astype(int)].tolist() if len(cand) else [])
    idx = np.array(sorted(set(pick)), dtype=np.int64)
    sub = tb.take(idx)
    planted = flatten_trees([parse_expression(e, opts) for e in ("x1 * 1.0e30", "x1 * 5.0e34", "(x2 * 4.0e34) + x3",
                                                                   "cos(x1) * 2.0e33")], np.float32)
    pl_loss, pl_comp = device_call(planted)
    X, y = c4_shard(0, 1, rows_total)
    orc = Oracle.from_options(opts)
    out = {}
    for name, t, d_loss, d_comp in (("sample", sub, np.asarray(res["l"])[idx], comp[idx]),
                                    ("planted_big", planted, pl_loss, pl_comp)):
        progress(f"c4 parity: oracle f64 sums of {name} ({t.n_trees} trees)")
        l64, c64 = orc.eval_loss_batch(t, X, y, accum="f64", n_threads=threads)
        progress(f"c4 parity: oracle in-order folds of {name}")
        lref, cref = orc.eval_loss_batch(t, X, y, accum="ref", n_threads=threads)
        progress(f"c4 parity: per-tree bars of {name}")
        d_loss = np.asarray(d_loss, dtype=np.float64)
        ok = d_comp & c64
        lr = (lref if accum == "ref" else l64).astype(np.float64)
        fin = ok & np.isfinite(lr)
        r, bar, err, n_wide = per_tree_bar(orc, t, X, y, d_loss, lr, fin, 1e-4, threads, accum=accum)
        fail = fin & ~(err <= bar)
        inf_m = int(np.sum(ok & (np.isinf(d_loss) != np.isinf(lref))))
        with np.errstate(invalid="ignore", divide="ignore"):
            r64 = np.where(d_loss == l64, 0.0, np.abs(d_loss - l64) / np.maximum(np.abs(l64.astype(np.float64)), 1e-300))
            lrf = lref.astype(np.float64)
            rrf = np.where(d_loss == lrf, 0.0, np.abs(d_loss - lrf) / np.maximum(np.abs(lrf), 1e-300))
        fin_r = fin & np.isfinite(lrf)
        out[name] = {"trees": int(t.n_trees), "complete": int(ok.sum()),
                     "flag_mismatches": int(np.sum(d_comp != c64)) + int(np.sum(cref != c64)),
                     "ref_fold_inf_trees": int(np.sum(ok & np.isinf(lref))), "ref_fold_inf_mismatches": inf_m,
                     ("n_bit_exact_vs_ref_f32_fold" if accum == "ref" else "n_bit_exact_vs_f64_accum"):
                         int(np.sum(fin & (d_loss.astype(np.float32) == lr.astype(np.float32)))),
                     ("max_rel_vs_ref_f32_fold" if accum == "ref" else "max_rel_vs_oracle"):
                         float(np.max(np.where(np.isfinite(r[fin]), r[fin], 0.0), initial=0.0)),
                     "max_rel_vs_f64_accum": float(np.max(np.where(np.isfinite(r64[fin]), r64[fin], 0.0), initial=0.0)),
                     # (the reference's own Float32 fold, whatever the device accumulated: at 2^26 rows it
                     #  stalls far below the exact mean)
                     "max_rel_device_vs_ref_f32_fold": float(np.max(np.where(np.isfinite(rrf[fin_r]), rrf[fin_r], 0.0),
                                                                    initial=0.0)),
                     "n_held_to_libm_spread_bar": n_wide, "loss_failures": int(fail.sum()),
                     "held_trees": held_trees(opts, orc, t, X, y, np.nonzero(fin & (r > 1e-4))[0], d_loss,
                                              lr, bar, threads, ids=idx if name == "sample" else None,
                                              accum=accum, limit=8)}
    out["rows"] = int(rows_total)
    out["accumulation"] = accum
    out["pass"] = all(v["flag_mismatches"] == 0 and v["loss_failures"] == 0 and v["ref_fold_inf_mismatches"] == 0
                      for v in (out["sample"], out["planted_big"]))
    out["rule"] = ("flags bit-exact vs the oracle over all rows; +Inf exactly where the reference's Float32 fold is; "
                   "complete losses within max(1e-4 |oracle|, 4 x libm spread) of the reference's in-order Float32 "
                   "fold (the oracle's accum='ref'); sample = the timed step's own "
                   "results for a stratified tree sample (3/4 complete, 1/4 incomplete, evenly over tree size); "
                   "planted_big = trees over values >= floatmax/2n (the exact Julia-order isfinite(sum) pass), "
                   "scored by the same sharded call")
    out["cpu_s"] = time.perf_counter() - t0
    return out


def extra_lines(ctx, opts, trees, comp, X, y, args):
    """The same C2 population (i) restricted to its complete trees — the interpreter's roofline
    without dead-tree skipping — and (ii) in Float64 against the FP64 peak, each with its per-launch
    breakdown (trees per workgroup G, workgroups, per-chunk time)."""
    from sr_amd import Dataset, flatten_trees

    out = {}
    steps, warm = max(5, args.steps // 2), 3
    live = [t for t, c in zip(trees, comp) if c]
    tbc = flatten_trees(live, np.float32)
    dsc = Dataset(X, y)
    call, _ = single_gpu_call(ctx, tbc, dsc, opts)
    st = {}
    dt, _, kms = timed(lib_step(ctx, call, st), steps, warm, lambda: None)
    km = float(np.mean(kms))
    out["roofline_complete_only"] = roofline(
        float(X.shape[1]) * (tbc.n_operator_nodes + 3 * tbc.n_trees), km, PEAK_FP32_TFLOPS,
        busy_ms_per_step=float(np.mean(st["busy"][-steps:])),
        n_trees=tbc.n_trees, ms_per_step=dt / steps * 1e3,
        node_evals_per_s=float(tbc.n_nodes) * X.shape[1] * steps / dt,
        launches=chunk_groups(tbc.n_trees, X.shape[1], int(round(np.mean(st["launches"][-steps:]))),
                              ctx.last_rows_per_lane()),
        what="the C2 population's complete trees only (every tree runs every row)")
    dsc.free_device()
    X64, y64 = X.astype(np.float64), y.astype(np.float64)
    tb64 = flatten_trees(trees, np.float64)
    ds64 = Dataset(X64, y64)
    call, o64 = single_gpu_call(ctx, tb64, ds64, opts, np.float64)
    st = {}
    dt, _, kms = timed(lib_step(ctx, call, st), steps, warm, lambda: None)
    km = float(np.mean(kms))
    busy = float(np.mean(st["busy"][-steps:]))
    rpl64 = ctx.last_rows_per_lane()
    f64_parity = None
    if not args.no_cpu_baseline:
        f64_parity = f64_parity_sample(opts, tb64, X64, y64, o64)
    out["f64"] = roofline(
        float(X.shape[1]) * (tb64.n_operator_nodes + 3 * tb64.n_trees), busy, PEAK_FP64_TFLOPS,
        parity=f64_parity,
        kernel_sum_ms_per_step=km, ms_per_step=dt / steps * 1e3,
        kernel=(f"sr_tile_kernel<double,{rpl64},LOSS,gather=false,BASIC" + (",register stack>" if rpl64 == 8 else ">")),
        node_evals_per_s=float(tb64.n_nodes) * X.shape[1] * steps / dt,
        fraction_complete=float(np.mean(o64["comp"].astype(bool))),
        convention="achieved / frac from the device-busy time (union of the launch intervals), which fits in the step",
        what="the C2 population and data in Float64 (C5's element type)")
    ds64.free_device()
    return out


def f64_parity_sample(opts, tb64, X64, y64, o64, n=320):
    """The timed Float64 step against the oracle at full size (2^20 rows): a strided tree sample, flags
    bit-exact, every complete tree within the north-star f64 bar (1e-10 relative, or 4 x the tree's
    libm spread: tests/parity_util.py)."""
    from oracle import Oracle

    threads = min(int(os.environ.get("OMP_NUM_THREADS", "0")) or (os.cpu_count() or 1), 16)
    t0 = time.perf_counter()
    step = max(1, tb64.n_trees // n)
    idx = np.arange(0, tb64.n_trees, step)[:n]
    sub = tb64.take(idx)
    orc = Oracle.from_options(opts)
    l64, c64 = orc.eval_loss_batch(sub, X64, y64, accum="ref", n_threads=threads)
    d_loss = np.asarray(o64["loss"], dtype=np.float64)[idx]
    d_comp = np.asarray(o64["comp"]).astype(bool)[idx]
    ok = d_comp & c64
    r, bar, err, n_wide = per_tree_bar(orc, sub, X64, y64, d_loss, l64, ok, 1e-10, threads)
    fail = ok & ~(err <= bar)
    fin = ok & np.isfinite(r)
    return {"trees": int(sub.n_trees), "rows": int(X64.shape[1]), "complete": int(ok.sum()),
            "flag_mismatches": int(np.sum(d_comp != c64)), "loss_failures": int(fail.sum()),
            "max_rel": float(np.max(r[fin], initial=0.0)), "median_rel": float(np.median(r[fin])) if fin.any() else 0.0,
            "n_held_to_libm_spread_bar": n_wide, "pass": bool(np.all(d_comp == c64) and not fail.any()),
            "held_trees": held_trees(opts, orc, sub, X64, y64, np.nonzero(ok & (r > 1e-10))[0], d_loss, l64, bar,
                                     threads, ids=idx),
            "rule": ("flags bit-exact; every complete tree within max(1e-10 |oracle|, 4 x libm spread) of the "
                     "reference's in-order Float64 fold (the oracle's accum='ref')"),
            "cpu_s": time.perf_counter() - t0}


def algorithmic_bytes(nt, rows, n_launch, rows_per_lane=8, n_derived=0):
    """Bytes the interpreter launches of a step must read: every tree-group pass streams the X rows
    (5 features) and y, plus the derived columns (LOAD_DERIVED inputs, read from HBM by the trees that
    use them: with tree groups dealt round-robin every group holds users of nearly every column)."""
    n_passes = sum(-(-c // g) for c, g, _ in chunk_groups(nt, rows, n_launch, rows_per_lane))
    return float(n_passes) * (5 + 1 + n_derived) * float(rows) * 4.0


def chunk_groups(nt, rows, n_launch, rows_per_lane=8):
    """(trees, trees per workgroup G, workgroups) of each interpreter launch of a step, as
    csrc/sr_capi.cpp's run_batch / make_grid split them (2 launches: a first chunk of nt/6 trees)."""
    tiles = -(-rows // (64 * rows_per_lane))
    n_rb = -(-tiles // (-(-tiles // 256)))
    bounds = [0, nt // 6, nt] if n_launch == 2 else [nt * k // n_launch for k in range(n_launch + 1)]
    out = []
    for a, b in zip(bounds[:-1], bounds[1:]):
        c = b - a
        g = int(os.environ.get("SR_AMD_TREES_PER_BLOCK", "0"))
        if not g:
            g = 128
            while g > 4 and n_rb * (-(-c // g)) < 4096:
                g //= 2
        g = max(1, min(g, c))
        out.append((c, g, n_rb * (-(-c // g))))
    return out


def set_ref_fold(v, lanes=4):
    """The in-order loss fold on (1) or off (0: the f64 per-tree sums) for every scoring context of this
    process (the default context and the search's extra lanes)."""
    from sr_amd.device import get_lane_context

    for lane in range(lanes):
        get_lane_context(lane).set_tuning("ref_fold", int(v))


def search_lines(args):
    """BASELINE.json metric, second half: search iterations/sec of C1 (the README example) and C3
    (Feynman-style 5-feature target, 100k rows, f32), device-scored, each beside the same engine with
    the same seeds scored by the C port on the host cores (`sr_search_use_callbacks` with the
    oracle's C scorers: a "port" CPU baseline)."""
    from oracle import Oracle, SearchScorer

    from sr_amd import Options, equation_search

    threads = min(int(os.environ.get("OMP_NUM_THREADS", "0")) or (os.cpu_count() or 1), 16)
    out = {}
    rng = np.random.default_rng(0)
    X1 = rng.standard_normal((2, 100))
    y1 = 2 * np.cos(X1[1]) + X1[0] ** 2 - 2
    o1 = Options(binary_operators=["+", "*", "/", "-"], unary_operators=["cos", "exp"], populations=20)
    rng = np.random.default_rng(11)
    X3 = rng.uniform(0.5, 2.0, (5, 100_000)).astype(np.float32)
    y3 = (X3[0] * X3[1] * X3[2] / (X3[3] * X3[4] ** 2 + 1)).astype(np.float32)
    o3 = Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp", "log"], populations=31)
    # C5: the C3 data in Float64, constant optimisation on (BFGS / Newton with the device's forward-mode
    # gradients; it is on by default, optimizer_probability 0.14), populations a multiple of 8
    X5, y5 = X3.astype(np.float64), y3.astype(np.float64)
    o5 = Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp", "log"], populations=32,
                 should_optimize_constants=True)
    for name, X, y, o, cpu_iters, cpu_threads, desc in (
            ("c1", X1, y1, o1, args.search_cpu_iters or args.search_iters, threads,
             "C1 README example: X=randn(2,100) f64, ops + * / - cos exp, 20 populations, default options"),
            ("c3", X3, y3, o3, args.search_cpu_iters or 2, threads,
             "C3: y = x1 x2 x3 / (x4 x5^2 + 1), X ~ U(0.5, 2) 5 x 100k f32, 31 populations, default options"),
            ("c5", X5, y5, o5, args.search_cpu_iters or 1, threads,
             "C5: the C3 data in f64, constant optimisation (BFGS / Newton, device forward-mode gradients), "
             "32 populations, default options")):
        progress(f"search {name}")
        t0 = time.perf_counter()
        res = equation_search(X, y, niterations=args.search_iters, options=o, seed=0)
        wall = time.perf_counter() - t0
        # per-call breakdown from a short second run with the kernel timing on (reading the events
        # costs every call their queries, so the timed run above goes without)
        os.environ["SR_AMD_SEARCH_KERNEL_TIMES"] = "1"
        diag = equation_search(X, y, niterations=min(5, args.search_iters), options=o, seed=0)
        del os.environ["SR_AMD_SEARCH_KERNEL_TIMES"]
        # the fold's cost: the same search scored with the f64 per-tree sums
        set_ref_fold(0)
        t0 = time.perf_counter()
        res0 = equation_search(X, y, niterations=args.search_iters, options=o, seed=0)
        wall0 = time.perf_counter() - t0
        set_ref_fold(1)
        line = {"metric": "search iterations/sec", "value": res.s_r_cycles / wall, "unit": "s_r_cycles/s",
                "loss_accumulation": "the reference's in-order fold in T (ref_fold 1, the default)",
                "iterations_per_s_f64_sum": args.search_iters / wall0,
                "device_wall_per_call_us_f64_sum": res0.device_s / max(res0.device_calls, 1) * 1e6,
                "iterations_per_s": args.search_iters / wall, "islands": o.populations,
                "iterations": args.search_iters, "wall_s": wall, "device_calls": res.device_calls,
                "device_wall_s": res.device_s, "host_s": res.host_s,
                "device_wall_per_call_us": res.device_s / max(res.device_calls, 1) * 1e6,
                "kernel_busy_per_call_us": diag.kernel_s / max(diag.device_calls, 1) * 1e6,
                "per_call_note": ("device_wall = wall time inside the scoring calls (the default four scoring lanes overlap); "
                                  "kernel_busy = the interpreter launches' device-busy time (a 5-iteration run "
                                  "with SR_AMD_SEARCH_KERNEL_TIMES=1)"),
                "best_loss": float(min(m.loss for m in res.pareto_frontier)), "config": desc}
        if name == "c5":
            line["grad_roofline"] = grad_roofline(res, X, y, o)
            # island sharding at 8 ranks: rank 0's share (islands i % 8 == 0, 4 of 32) —
            # its islands' rounds and constant optimisation on its own GPU, the head over all islands —
            # measured in one process without the per-iteration island exchange (a few KB all-gather)
            progress("search c5: rank 0's share of an 8-rank island-sharded search")
            share = equation_search(X, y, niterations=args.search_iters, options=o, seed=0, _rank_share=(0, 8))
            swall = share.wall_s  # (the search loop; the helper engines' start is before it)
            rate32, rate4 = args.search_iters / res.wall_s, args.search_iters / swall
            # weak scaling (the north star's "island populations sharded": more islands per job): 8 ranks
            # x 32 islands = 256, rank 0's 32 own islands and the head over all 256
            import copy
            o256 = copy.copy(o)
            o256.populations = 8 * o.populations
            progress("search c5: rank 0's share of an 8-rank search with 8x the islands (weak scaling)")
            weak = equation_search(X, y, niterations=args.search_iters, options=o256, seed=0, _rank_share=(0, 8))
            rate_w = args.search_iters / weak.wall_s
            line["projection_8_ranks"] = {
                "rank0_islands": len(range(0, o.populations, 8)), "rank0_iterations_per_s": rate4,
                "rank0_device_calls": share.device_calls, "one_gpu_iterations_per_s": rate32,
                "speedup": rate4 / rate32, "efficiency": rate4 / rate32 / 8.0,
                "weak_scaling": {"islands_total": o256.populations, "rank0_islands": len(range(0, o256.populations, 8)),
                                 "rank0_iterations_per_s": rate_w, "efficiency": rate_w / rate32,
                                 "note": ("8 ranks x the one-GPU island count: the job runs 8x the islands at rank "
                                          "0's rate; efficiency = that rate / the one-GPU 32-island rate")},
                "model": ("the 8-rank search runs at the rate of its slowest rank; rank 0's share measured alone "
                          "(equation_search(_rank_share=(0, 8)): its 4 islands' regularised-evolution rounds and "
                          "constant optimisation, the other islands imported every iteration as initialised, the "
                          "head over all 32 islands), without the all-gather itself; rates from the search loops' "
                          "own wall clocks")}
        sc = SearchScorer(Oracle.from_options(o), X, y, n_threads=cpu_threads)
        t0 = time.perf_counter()
        cres = equation_search(X, y, niterations=cpu_iters, options=o, seed=0, _native_scorer=sc)
        cwall = time.perf_counter() - t0
        line["cpu_baseline"] = {
            "value": cres.s_r_cycles / cwall, "unit": "s_r_cycles/s", "iterations_per_s": cpu_iters / cwall,
            "cores": cpu_threads, "kind": "port",
            "sample": (f"the same engine and seeds, every scoring call answered by the C oracle on {cpu_threads} host "
                       f"core(s) (loss folded in T; gradients by central differences as the reference's Optim "
                       f"BFGS), {cpu_iters} iteration(s), {cwall:.1f} s, {cres.device_calls} scoring calls")}
        out[name] = line
    return out


def grad_roofline(res, X, y, opts, reps=5):
    """The gradient kernel (sr_eval_grad_batch: BFGS's objective + gradient, src/ConstantOptimization.jl:
    126-167) on the C5 search's final members with constants, over the full data: per tangent bucket the
    tangent kernel's HIP-event time and its algorithmic flops (csrc sr_last_grad_info: per row and work
    item, each unary node 2 + KT, binary node 3 + 2 KT, loss epilogue 3 + KT), against the FP64 peak."""
    from sr_amd import flatten_trees

    trees = [m.tree for p in res.populations for m in p if m.tree.count_constants() > 0]
    return grad_roofline_batch(flatten_trees(trees, np.float64), X, y, opts, reps)


def grad_roofline_batch(tb, X, y, opts, reps=5):
    """grad_roofline's measurement on a flattened batch (tools/c5_grad_profile.py profiles it alone)."""
    import sr_amd
    from sr_amd import Dataset, eval_grad_batch

    ds = Dataset(X, y)
    ctx = sr_amd.get_context()
    for _ in range(2):
        eval_grad_batch(tb, ds, opts)
    per = None
    for _ in range(reps):
        eval_grad_batch(tb, ds, opts)
        info = ctx.last_grad_info()
        if per is None:
            per = [dict(b, kernel_ms=0.0) for b in info]
        for a, b in zip(per, info):
            a["kernel_ms"] += b["kernel_ms"] / reps
    buckets = []
    for b in per:
        if b["items"] == 0:
            continue
        ach = b["flops"] / (b["kernel_ms"] * 1e-3) / 1e12 if b["kernel_ms"] > 0 else 0.0
        buckets.append(dict(b, achieved_TFLOPs=ach, frac=ach / PEAK_FP64_TFLOPS))
    tot_ms = sum(b["kernel_ms"] for b in buckets)
    tot_fl = sum(b["flops"] for b in buckets)
    dom = max(buckets, key=lambda b: b["kernel_ms"]) if buckets else None
    ach = tot_fl / (tot_ms * 1e-3) / 1e12 if tot_ms > 0 else 0.0
    ds.free_device()
    return {"bound": "valu", "achieved": ach, "peak": PEAK_FP64_TFLOPS, "unit": "TFLOP/s", "frac": ach / PEAK_FP64_TFLOPS,
            "kernel_ms_per_call": tot_ms, "flops_per_call": tot_fl, "dominant_bucket": dom, "buckets": buckets,
            "trees": int(tb.n_trees), "rows": int(X.shape[1]), "dtype": "f64",
            "kernel": "sr_grad_kernel<double,KT,W=4,gather=false,R>",
            "flop_convention": ("per row and (tree, first tangent) item: unary node 2 + KT, binary node 3 + 2 KT, "
                                "loss epilogue 3 + KT; 1 flop per operator incl. transcendentals"),
            "what": "sr_eval_grad_batch on the C5 search's final members with constants, full 100k rows, f64"}


def measured_traffic(workload, n_trees, rows_per_gpu):
    """Per-step HBM bytes of the interpreter from the committed rocprofv3 PMC pass of this same
    command (profiles/traffic.json / traffic_c4.json, written by tools/trace_frac.py) — only when it
    was measured on this configuration (files without the configuration: the default one)."""
    p = os.path.join(ROOT, "profiles", "traffic.json" if workload == "c2" else f"traffic_{workload}.json")
    try:
        with open(p) as f:
            t = json.load(f)
    except (OSError, ValueError):
        return None
    if t.get("workload") != workload or "hbm_read_bytes_per_step" not in t:
        return None
    default = (10_000, 1 << 20) if workload == "c2" else (100_000, 1 << 26)
    if (t.get("n_trees", default[0]), t.get("rows_per_gpu", default[1])) != (n_trees, rows_per_gpu):
        return None
    t["source"] = (f"profiles/{os.path.basename(p)} (rocprofv3 --pmc FETCH_SIZE of the bench command, "
                   "x1024 B x2 gfx950, the timed steps' interpreter launches)")
    return t


def cpu_baseline_and_parity(opts, tb, X, y, n_sample, dev_loss, dev_comp):
    """CPU baseline: the oracle (C port of DE's array-at-a-time evaluator, OpenMP over trees) on a
    bounded sample — a strided subset of the same trees over the same 1M rows (~15 s on <= 16 host
    cores), timed with the reference's sequential Float32 loss fold.
    Parity of the TIMED step on that sample: flags bit-exact; every complete tree's loss within the
    per-tree bar (1e-4 relative, or 4x the tree's own spread under +-1-ulp libm perturbations — the
    tests' rule) of the reference's sequential Float32 fold (the device's loss IS that fold)."""
    from oracle import Oracle

    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(os.cpu_count() or 1, 16)
    threads = min(threads, 16)
    orc = Oracle.from_options(opts)

    def pick(n):
        step = max(1, tb.n_trees // n)
        idx = np.arange(0, tb.n_trees, step)[:n]
        return idx, tb.take(idx), step

    def run(n):
        idx, sub, step = pick(n)
        t0 = time.perf_counter()
        l, c = orc.eval_loss_batch(sub, X, y, accum="ref", n_threads=threads)
        return idx, sub, step, time.perf_counter() - t0, l, c

    if n_sample <= 0:  # pilot, then size the sample for ~15 s of CPU work
        _, _, _, dt, _, _ = run(2 * threads)
        n_sample = int(min(tb.n_trees, max(2 * threads, 2 * threads * 15.0 / max(dt, 1e-3))))
    idx, sub, step, dt, l_ref, c_ref = run(n_sample)
    rate = float(sub.n_nodes) * X.shape[1] / dt
    cpu = {"value": rate, "unit": "node-evals/s", "cores": threads, "kind": "port",
           "sample": f"{sub.n_trees} of {tb.n_trees} trees (every {step}th), {X.shape[1]} rows, {dt:.1f} s"}

    l_f64, c_f64 = orc.eval_loss_batch(sub, X, y, accum="f64", n_threads=threads)
    d_loss, d_comp = dev_loss[idx].astype(np.float64), dev_comp[idx]
    flag_mismatch = int(np.sum(d_comp != c_ref)) + int(np.sum(c_ref != c_f64))
    ok = d_comp & c_ref
    lr = l_ref.astype(np.float64)
    l64 = l_f64.astype(np.float64)
    # the reference's L(Inf) where its Float32 loss fold overflows (src/LossFunctions.jl:38-58): the
    # device must be +Inf exactly there
    inf_mism = int(np.sum(ok & (np.isinf(d_loss) != np.isinf(l_ref))))
    n_fold_inf = int(np.sum(ok & np.isinf(l_ref)))
    fin = ok & np.isfinite(lr)
    # every complete tree's loss is the reference's in-order fold in T (round 6): against the oracle's
    # fold of its OWN element losses the difference left is the libm last-bit spread only, so the bar is
    # the tests' per-tree bar (1e-4, or 4 x the tree's spread under +-1-ulp libm perturbations)
    rref, bar, errref, n_wide = per_tree_bar(orc, sub, X, y, d_loss, lr, fin, 1e-4, threads)
    failref = fin & ~(errref <= bar)
    n_exact = int(np.sum(fin & (d_loss.astype(np.float32) == l_ref)))
    with np.errstate(invalid="ignore", divide="ignore"):
        r64 = np.where(d_loss == l64, 0.0, np.abs(d_loss - l64) / np.maximum(np.abs(l64), 1e-30))
        rfold = np.where(lr == l64, 0.0, np.abs(lr - l64) / np.maximum(np.abs(l64), 1e-30))
    fin64 = fin & np.isfinite(l64)
    parity = {"sample": cpu["sample"], "trees": int(sub.n_trees), "rows": int(X.shape[1]),
              "accumulation": "the reference's in-order fold in Float32 (LossFunctions.jl:38-58; oracle accum='ref')",
              "flags_bit_exact": flag_mismatch == 0, "flag_mismatches": flag_mismatch,
              "complete": int(ok.sum()),
              "n_bit_exact_vs_ref_f32_fold": n_exact,
              "max_rel_vs_ref_f32_fold": float(np.max(np.where(np.isfinite(rref[fin]), rref[fin], 0.0), initial=0.0)),
              "median_rel_vs_ref_f32_fold": float(np.median(rref[fin])) if fin.any() else 0.0,
              "n_held_to_libm_spread_bar": n_wide,
              "held_trees": held_trees(opts, orc, sub, X, y, np.nonzero(fin & (rref > 1e-4))[0], d_loss, lr, bar,
                                       threads, ids=idx),
              "loss_failures_vs_ref_fold": int(failref.sum()),
              "ref_fold_inf_trees": n_fold_inf,
              "ref_fold_inf_mismatches": inf_mism,
              # (information: the f64-accumulated sum is NOT the reference's loss; at 2^20 rows the fold's
              #  own rounding is ~1e-4 relative)
              "max_rel_vs_f64_accum": float(np.max(r64[fin64], initial=0.0)),
              "median_rel_vs_f64_accum": float(np.median(r64[fin64])) if fin64.any() else 0.0,
              "ref_f32_fold_self_error_median_rel": float(np.median(rfold[fin64])) if fin64.any() else 0.0,
              "ref_f32_fold_self_error_max_rel": float(np.max(rfold[fin64], initial=0.0)),
              "pass": flag_mismatch == 0 and not failref.any() and inf_mism == 0,
              "rule": ("flags bit-exact; +Inf exactly where the reference's sequential Float32 loss fold overflows; "
                       "every complete tree within max(1e-4 |oracle|, 4 x the tree's libm spread) of the reference's "
                       "in-order Float32 fold (tests/parity_util.py); bit-exact whenever the device's element losses "
                       "are (tests/test_gpu_ref_fold.py)")}
    return cpu, parity


if __name__ == "__main__":
    main()
