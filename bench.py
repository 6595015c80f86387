#!/usr/bin/env python3
"""Benchmark: batched eval_loss throughput (BASELINE.json metric) on C2 (default) or C4.

One step = score the whole population once: compile the trees into device programs, upload, run
the interpreter over all rows, reduce, copy losses back, exact re-check when needed, finalize (the
full cost of one `eval_cost_batch` call of a search iteration).  Trees and data are synthetic
(seeded), generated before timing; the dataset is resident in HBM when the timed region starts.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c2|c4]

c2 (default): BASELINE config 2, 10k trees x 1M rows x 5 features per GPU.  N > 1 (launched by
  torch.distributed.run): weak scaling — every rank holds its own 1M-row shard of one N x 1M-row
  dataset; the ranks combine per-tree partials with ONE all-reduce of a packed device buffer.
c4: BASELINE config 4, 100k trees x 64M rows (2^26) x 5 features, FIXED total rows sharded n/N
  over the N ranks (strong scaling: the configuration the 85 % scaling target is quoted on).

Rank 0 prints one JSON line.  Beside the headline it reports the interpreter's roofline (HIP-event
kernel time on the library's streams), the same population restricted to its complete trees
(no dead-tree skipping can flatter it), the population in Float64 (C5's type, against the FP64
peak), the CPU baseline (the C oracle on the host's cores) and the C1 search throughput.
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "symbolicregression.jl_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import sr_amd  # noqa: E402
from sr_amd import Dataset, Options, _lib, flatten_trees, gen_random_population  # noqa: E402

PEAK_FP32_TFLOPS = 157.3  # MI355X FP32 vector dense peak (packed FMA), MI355X_MICROARCH.md
PEAK_FP64_TFLOPS = 78.6   # MI355X FP64 vector dense peak
C2_OPS = dict(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp", "log"])
BLOCK = 1 << 20           # C4 data is generated in seeded 1M-row blocks (shards are whole blocks)


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
    return X, y, b0 * BLOCK


def timed(step, steps, warmup, barrier):
    """W untimed steps, then K timed steps between barriers (+ device sync)."""
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


def single_gpu_step(ctx, tb, ds, opts, dtype=np.float32):
    """One sr_eval_loss_batch over the whole population -> its interpreter time (ms)."""
    dsh = ds.device_handle(ctx)
    oid = ctx.opset_id(opts.operators)
    s = tb.to_struct()
    losses = np.empty(tb.n_trees, dtype=dtype)
    comp = np.empty(tb.n_trees, dtype=np.uint8)
    state = {"launches": []}

    def step():
        _lib.check(_lib.lib.sr_eval_loss_batch(ctx.handle, dsh, oid, ctypes.byref(s), None, 0, 0,
                                               losses.ctypes.data_as(ctypes.c_void_p),
                                               comp.ctypes.data_as(ctypes.c_void_p)))
        state["launches"].append(ctx.last_launches())
        return ctx.last_kernel_ms()[0]

    return step, losses, comp, state


def roofline(flops, kernel_ms, peak, **extra):
    achieved = flops / (kernel_ms * 1e-3) / 1e12
    out = {"bound": "valu", "achieved": achieved, "peak": peak, "unit": "TFLOP/s", "frac": achieved / peak,
           "kernel_ms_per_step": kernel_ms, "flops_per_step": flops}
    out.update(extra)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=8)
    ap.add_argument("--workload", choices=["c2", "c4"], default="c2")
    ap.add_argument("--rows", type=int, default=0, help="c2: rows per GPU (default 2^20); c4: total rows (2^26)")
    ap.add_argument("--trees", type=int, default=0, help="default 10k (c2) / 100k (c4)")
    ap.add_argument("--cpu-trees", type=int, default=0, help="CPU-baseline tree sample (0 = auto)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extra", action="store_true", help="skip the complete-only and Float64 lines")
    ap.add_argument("--search-iters", type=int, default=40,
                    help="iterations of the C1 search for the 'search iterations/sec' figure (0 = skip)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    # SR_BENCH_FORCE_DIST=1 (under torch.distributed.run): the multi-GPU code path at world size 1
    # (rehearses the scaling run's rendezvous, RCCL communicator and sharded step on one GPU)
    if world > 1 or os.environ.get("SR_BENCH_FORCE_DIST") == "1":
        import torch.distributed as tdist

        # gloo (CPU) for the rendezvous, the barrier and the max-over-ranks timing; the data path's
        # exchange is the library's own RCCL all-reduce over xGMI (sr_comm_*): torch's bundled HIP
        # runtime cannot share a GPU with the library's in one process, so torch never touches it
        tdist.init_process_group(backend="gloo")
        dist = tdist
    c4 = args.workload == "c4"
    if c4 and args.steps == 20 and args.warmup == 8:  # a C4 step is ~2 s on one GPU: fewer by default
        args.steps, args.warmup = 5, 2

    opts = Options(**C2_OPS)
    nt = args.trees or (100_000 if c4 else 10_000)
    trees = gen_random_population(nt, opts, 5, max_size=30, seed=4 if c4 else 1)
    tb = flatten_trees(trees, np.float32)
    if c4:
        rows_total = args.rows or (1 << 26)
        if rows_total % (BLOCK * world):
            raise SystemExit("c4: total rows must be a multiple of 2^20 x N")
        X, y, _ = c4_shard(rank, world, rows_total)
    else:
        rows_total = (args.rows or (1 << 20)) * world
        X, y = c2_data(rows_total // world, rank)
    n_local = X.shape[1]
    ctx = sr_amd.get_context(local_rank)
    if dist is not None:
        from sr_amd.distributed import init_device_comm

        init_device_comm(ctx=ctx)
    ds = Dataset(X, y)
    ds.device_handle(ctx)  # upload before timing

    if dist is None:
        step, losses, comp, state = single_gpu_step(ctx, tb, ds, opts)

        def barrier():
            pass
    else:
        from sr_amd.distributed import eval_loss_sharded

        result, state = {}, {"launches": []}

        def step():
            result["loss"], result["comp"] = eval_loss_sharded(tb, ds, opts, rows_total)
            state["launches"].append(ctx.last_launches())
            return ctx.last_kernel_ms()[0]

        def barrier():
            # every library call returns after its stream has drained (device synchronised)
            dist.barrier()

    dt, step_ms, kernel_ms = timed(step, args.steps, args.warmup, barrier)
    if dist is not None:
        import torch

        tt = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
        comp = result["comp"]

    nodes, ops = int(tb.n_nodes), int(tb.n_operator_nodes)
    node_evals = float(nodes) * float(rows_total)  # all ranks
    value = node_evals * args.steps / dt
    kmean = float(np.mean(kernel_ms))
    n_launch = int(round(float(np.mean(state["launches"][-args.steps:])))) if state["launches"] else 1
    flops_per_step = float(n_local) * (ops + 3 * nt)  # this GPU's interpreter work per step
    traffic = measured_traffic(args.workload)
    rpl = ctx.last_rows_per_lane()  # the interpreter build the library picked for this view
    frac_complete = float(np.mean(np.asarray(comp).astype(bool)))

    extra = {}
    if rank == 0 and world == 1 and not args.no_extra and not c4:
        extra = extra_lines(ctx, opts, trees, np.asarray(comp).astype(bool), X, y, args)
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(opts, tb, X[:, :min(n_local, 1 << 20)], y[:min(n_local, 1 << 20)], args.cpu_trees)
    search = None
    if rank == 0 and world == 1 and args.search_iters > 0 and not c4:
        search = search_throughput(args.search_iters)

    if rank == 0:
        if c4:
            workload = (f"C4 row-sharded eval_loss: {nt // 1000}k random trees (size U{{1..30}}; +,-,*,/,cos,exp,"
                        f"safe_log) x {rows_total >> 20}M rows x 5 features, rows sharded n/{world}")
        else:
            workload = (f"C2 batched eval_loss: {nt // 1000}k random trees (size U{{1..30}}; +,-,*,/,cos,exp,safe_log)"
                        f" x {n_local >> 20}M rows x 5 features per GPU")
        line = {
            "metric": "tree-node x row evals/sec (batched eval_loss, fp32)",
            "value": value,
            "unit": "node-evals/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": dt / args.steps * 1e3,
            "step_ms_min_median_max": [float(step_ms.min()), float(np.median(step_ms)), float(step_ms.max())],
            "higher_is_better": True,
            "scaling": "strong" if c4 else "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (seeded): gen_random_tree_fixed_size population, X~N(0,1), y=2cos(x4)+x1^2-2+0.1N",
            "config": {
                "workload": workload,
                "n_trees": nt,
                "tree_nodes": nodes,
                "operator_nodes": ops,
                "rows_per_gpu": n_local,
                "rows_total": rows_total,
                "nfeatures": 5,
                "parallelism": (f"rows sharded x{world}; one RCCL all-reduce of packed [4, n_trees] per-tree partials"
                                if world > 1 else "single GPU"),
                "fraction_complete": frac_complete,
            },
            "roofline": roofline(
                flops_per_step, kmean, PEAK_FP32_TFLOPS,
                traffic=traffic.get("hbm_read_bytes_per_step") if traffic else None,
                traffic_source=traffic.get("source") if traffic else None,
                kernel=(f"sr_tile_kernel<float,{rpl},LOSS,gather=false,BASIC,W=4,L2"
                        + (",register stack>" if rpl >= 16 else ">")),
                launches_per_step=n_launch,
                kernel_ms_convention=("per step: sum of the interpreter launches' HIP-event durations on the "
                                      "library's streams (= the kernel-trace sum: overlapping chunks count fully)"),
                flop_convention="n_rows * sum_t(n_op(t) + 3), 1 flop per operator incl. transcendentals (SURVEY 8d)",
                algorithmic_bytes_per_step=algorithmic_bytes(nt, n_local, n_launch, rpl),
                bytes_convention="ceil(n_trees/G) passes x (nf+1) x n_rows x 4 B; X/y re-reads are served from L2/MALL",
            ),
            "cpu_baseline": cpu,
            "search": search,
        }
        line["roofline"]["algorithmic_GBps"] = line["roofline"]["algorithmic_bytes_per_step"] / (kmean * 1e-3) / 1e9
        line.update(extra)
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def extra_lines(ctx, opts, trees, comp, X, y, args):
    """The same C2 population (i) restricted to its complete trees — the interpreter's roofline
    without dead-tree skipping — and (ii) in Float64 against the FP64 vector peak."""
    out = {}
    steps, warm = max(5, args.steps // 2), 3
    live = [t for t, c in zip(trees, comp) if c]
    tbc = flatten_trees(live, np.float32)
    dsc = Dataset(X, y)
    step, _, _, _ = single_gpu_step(ctx, tbc, dsc, opts)
    dt, _, kms = timed(step, steps, warm, lambda: None)
    km = float(np.mean(kms))
    out["roofline_complete_only"] = roofline(
        float(X.shape[1]) * (tbc.n_operator_nodes + 3 * tbc.n_trees), km, PEAK_FP32_TFLOPS,
        n_trees=tbc.n_trees, ms_per_step=dt / steps * 1e3,
        node_evals_per_s=float(tbc.n_nodes) * X.shape[1] * steps / dt,
        what="the C2 population's complete trees only (every tree runs every row)")
    dsc.free_device()
    X64, y64 = X.astype(np.float64), y.astype(np.float64)
    tb64 = flatten_trees(trees, np.float64)
    ds64 = Dataset(X64, y64)
    step, _, c64, _ = single_gpu_step(ctx, tb64, ds64, opts, np.float64)
    dt, _, kms = timed(step, steps, warm, lambda: None)
    km = float(np.mean(kms))
    out["f64"] = roofline(
        float(X.shape[1]) * (tb64.n_operator_nodes + 3 * tb64.n_trees), km, PEAK_FP64_TFLOPS,
        kernel="sr_tile_kernel<double,4,LOSS,gather=false,BASIC>", ms_per_step=dt / steps * 1e3,
        node_evals_per_s=float(tb64.n_nodes) * X.shape[1] * steps / dt,
        fraction_complete=float(np.mean(c64.astype(bool))),
        what="the C2 population and data in Float64 (C5's element type)")
    ds64.free_device()
    return out


def algorithmic_bytes(nt, rows, n_launch, rows_per_lane=8):
    n_passes = sum(-(-c // g) for c, g in chunk_groups(nt, rows, n_launch, rows_per_lane))
    return float(n_passes) * (5 + 1) * float(rows) * 4.0


def chunk_groups(nt, rows, n_launch, rows_per_lane=8):
    """(trees, trees per workgroup) of each interpreter launch of a step, as csrc/sr_capi.cpp's
    run_batch / make_grid split them (2 launches: a first chunk of nt/6 trees)."""
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
        out.append((c, max(1, min(g, c))))
    return out


def search_throughput(niterations):
    """BASELINE.json metric, second half: search iterations/sec on C1 (README example: X = randn(2, 100)
    f64, ops + * / - cos exp, 20 populations, default options, 40 iterations), lock-step islands with
    one batched device scoring call per evolution round (sr_amd.search.equation_search).
    Iterations/sec counts completed s_r_cycles (one per island per iteration,
    src/SymbolicRegression.jl:1091) per wall second."""
    from sr_amd import equation_search

    rng = np.random.default_rng(0)
    Xs = rng.standard_normal((2, 100))
    ys = 2 * np.cos(Xs[1]) + Xs[0] ** 2 - 2
    sopts = Options(binary_operators=["+", "*", "/", "-"], unary_operators=["cos", "exp"], populations=20)
    t0 = time.perf_counter()
    res = equation_search(Xs, ys, niterations=niterations, options=sopts, seed=0)
    wall = time.perf_counter() - t0
    return {"metric": "search iterations/sec", "value": res.s_r_cycles / wall, "unit": "s_r_cycles/s",
            "iterations_per_s": niterations / wall, "islands": sopts.populations, "iterations": niterations,
            "wall_s": wall, "device_calls": res.device_calls,
            "best_loss": float(min(m.loss for m in res.pareto_frontier)),
            "config": "C1 README example, X=randn(2,100) f64, 20 populations, default options",
            "cpu_baseline": None,
            "cpu_baseline_note": "the reference's Julia search cannot run here (no Julia runtime in the image)"}


def measured_traffic(workload):
    """Per-step HBM bytes of the interpreter from the committed rocprofv3 PMC pass of this same
    command (profiles/traffic.json, written by tools/trace_frac.py)."""
    p = os.path.join(ROOT, "profiles", "traffic.json")
    try:
        with open(p) as f:
            t = json.load(f)
    except (OSError, ValueError):
        return None
    if t.get("workload") != workload or "hbm_read_bytes_per_step" not in t:
        return None
    t["source"] = ("profiles/traffic.json (tools/bench_evidence.sh: rocprofv3 --pmc FETCH_SIZE of this bench "
                   "command, x1024 B x2 gfx950, the timed steps' interpreter launches)")
    return t


def cpu_baseline(opts, tb, X, y, n_sample):
    """Oracle (C port of DE's array-at-a-time evaluator, OpenMP over trees) on a bounded sample:
    a strided subset of the same trees over the first <= 1M rows (~10-30 s on 16 host cores)."""
    from oracle import Oracle

    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(os.cpu_count() or 1, 16)
    threads = min(threads, 16)
    orc = Oracle.from_options(opts)

    def run(n):
        step = max(1, tb.n_trees // n)
        sub = tb.subset(np.arange(0, tb.n_trees, step)[:n])
        t0 = time.perf_counter()
        orc.eval_loss_batch(sub, X, y, accum="ref", n_threads=threads)
        return sub, step, time.perf_counter() - t0

    if n_sample <= 0:  # pilot, then size the sample for ~15 s of CPU work
        sub, step, dt = run(2 * threads)
        n_sample = int(min(tb.n_trees, max(2 * threads, 2 * threads * 15.0 / max(dt, 1e-3))))
    sub, step, dt = run(n_sample)
    rate = float(sub.n_nodes) * X.shape[1] / dt
    return {
        "value": rate,
        "unit": "node-evals/s",
        "cores": threads,
        "kind": "port",
        "sample": f"{sub.n_trees} of {tb.n_trees} trees (every {step}th), {X.shape[1]} rows, {dt:.1f} s",
    }


if __name__ == "__main__":
    main()
