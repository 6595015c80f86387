#!/usr/bin/env python3
"""Benchmark: batched eval_loss throughput (BASELINE.json metric, config C2 / C4-style sharding).

One step = score the whole population once: compile the 10k trees into device programs, upload,
run the interpreter over all rows, reduce, copy losses back, finalize (the full cost of one
`eval_cost_batch` call of a search iteration).  Trees and data are synthetic (seeded), generated
before timing; the dataset is resident in HBM when the timed region starts.

  python bench.py [--gpus N] [--steps K] [--warmup W]
N > 1 (launched by torch.distributed.run): weak scaling — every rank holds its own 1M-row shard of
one N*1M-row dataset, computes per-tree partial Σloss + flags, and the ranks all-reduce them over
RCCL (the path's real exchange step) before finalizing.
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

PEAK_FP32_TFLOPS = 157.3  # MI355X FP32 vector (= FP32 MFMA) dense peak, MI355X_MICROARCH.md


def c2_workload(n_rows, n_trees, rank, nf=5):
    opts = Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp", "log"])
    trees = gen_random_population(n_trees, opts, nf, max_size=30, seed=1)
    tb = flatten_trees(trees, np.float32)
    rng = np.random.default_rng(2 + 1000 * rank)
    X = rng.standard_normal((nf, n_rows)).astype(np.float32)
    y = (2 * np.cos(X[3]) + X[0] ** 2 - 2 + 0.1 * np.random.default_rng(3 + 1000 * rank).standard_normal(n_rows)
         ).astype(np.float32)
    return opts, tb, X, y


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=8)
    ap.add_argument("--rows", type=int, default=1 << 20, help="rows per GPU")
    ap.add_argument("--trees", type=int, default=10000)
    ap.add_argument("--cpu-trees", type=int, default=0, help="CPU-baseline tree sample (0 = auto)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--search-iters", type=int, default=2,
                    help="iterations of the C1 search for the secondary 'search iterations/sec' figure (0 = skip)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as tdist

        torch.cuda.set_device(local_rank)
        tdist.init_process_group(backend="nccl")
        dist = tdist

    opts, tb, X, y = c2_workload(args.rows, args.trees, rank)
    n_total = args.rows * world
    ctx = sr_amd.get_context(local_rank)
    ds = Dataset(X, y)
    dsh = ds.device_handle(ctx)
    oid = ctx.opset_id(opts.operators)
    s = tb.to_struct()
    nt = tb.n_trees

    launches = []
    if world == 1:
        losses = np.empty(nt, dtype=np.float32)
        comp = np.empty(nt, dtype=np.uint8)

        def step():
            _lib.check(_lib.lib.sr_eval_loss_batch(ctx.handle, dsh, oid, ctypes.byref(s), None, 0, 0,
                                                   losses.ctypes.data_as(ctypes.c_void_p),
                                                   comp.ctypes.data_as(ctypes.c_void_p)))
            launches.append(ctx.last_launches())
            return ctx.last_kernel_ms()[0]

        def barrier():
            pass
    else:
        import torch

        from sr_amd.distributed import eval_loss_sharded

        result = {}

        def step():
            result["loss"], result["comp"] = eval_loss_sharded(tb, ds, opts, n_total)
            launches.append(ctx.last_launches())
            return ctx.last_kernel_ms()[0]

        def barrier():
            dist.barrier()
            torch.cuda.synchronize()

    for _ in range(args.warmup):
        step()
    barrier()
    kernel_ms, step_t = [], []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        kernel_ms.append(step())
        step_t.append(time.perf_counter())
    barrier()
    dt = time.perf_counter() - t0
    step_ms = np.diff(np.array([t0] + step_t)) * 1e3  # per-step wall (rank-local), jitter diagnostics
    if dist is not None:
        import torch

        tt = torch.tensor([dt], dtype=torch.float64, device=torch.device("cuda", local_rank))
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())

    nodes = int(tb.n_nodes)
    ops = int(tb.n_operator_nodes)
    node_evals = float(nodes) * float(n_total)            # all ranks
    value = node_evals * args.steps / dt
    # roofline of the interpreter kernel on this GPU: algorithmic flops of a step's interpreter work
    # / the step's interpreter time (Σ of its launch durations: the batch is compiled and launched in
    # `launches_per_step` chunks; a kernel trace's per-launch average x launches_per_step = kmean)
    flops_per_step = float(args.rows) * (ops + 3 * nt)
    kmean = float(np.mean(kernel_ms))
    n_launch = int(round(float(np.mean(launches[-args.steps:])))) if launches else 1
    achieved = flops_per_step / (kmean * 1e-3) / 1e12
    # algorithmic bytes: one pass of X + y per tree group of every launch
    n_passes = sum(-(-c // g) for c, g in chunk_groups(nt, args.rows, n_launch))
    bytes_per_step = float(n_passes) * (5 + 1) * float(args.rows) * 4.0
    traffic = measured_traffic()
    if world > 1:
        comp = result["comp"]
    frac_complete = float(np.mean(comp.astype(bool)))

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(opts, tb, X, y, args.cpu_trees)
    search = None
    if rank == 0 and world == 1 and args.search_iters > 0:
        search = search_throughput(args.search_iters)

    if rank == 0:
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
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (seeded): gen_random_tree_fixed_size population, X~N(0,1), y=2cos(x4)+x1^2-2+0.1N",
            "config": {
                "workload": "C2 batched eval_loss: 10k random trees (size U{1..30}; +,-,*,/,cos,exp,safe_log) x 1M rows x 5 features per GPU",
                "n_trees": nt,
                "tree_nodes": nodes,
                "operator_nodes": ops,
                "rows_per_gpu": args.rows,
                "rows_total": n_total,
                "nfeatures": 5,
                "parallelism": f"rows sharded x{world}, RCCL all-reduce of per-tree partial sums" if world > 1 else "single GPU",
                "fraction_complete": frac_complete,
            },
            "roofline": {
                "bound": "valu",
                "achieved": achieved,
                "peak": PEAK_FP32_TFLOPS,
                "unit": "TFLOP/s",
                "frac": achieved / PEAK_FP32_TFLOPS,
                "traffic": traffic.get("hbm_read_bytes_per_step") if traffic else None,
                "traffic_source": traffic.get("source") if traffic else None,
                "kernel": "sr_tile_kernel<float,8,LOSS,gather=false,BASIC>",
                "kernel_ms_mean": kmean,
                "launches_per_step": n_launch,
                "kernel_ms_convention": "per step: sum of the interpreter launches' HIP-event durations (library stream)",
                "flops_per_step": flops_per_step,
                "flop_convention": "n_rows * sum_t(n_op(t) + 3), 1 flop per operator incl. transcendentals (SURVEY 8d)",
                "algorithmic_bytes_per_step": bytes_per_step,
                "algorithmic_GBps": bytes_per_step / (kmean * 1e-3) / 1e9,
                "per_step": "achieved, traffic and bytes are per step (all launches of the step)",
                "bytes_convention": "ceil(n_trees/G) passes x (nf+1) x n_rows x 4 B; X/y re-reads are served from L2/MALL",
            },
            "cpu_baseline": cpu,
            "search": search,
        }
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def chunk_groups(nt, rows, n_launch):
    """(trees, trees per workgroup) of each interpreter launch of a step, as csrc/sr_capi.cpp's
    run_batch / make_grid split them (2 launches: a first chunk of nt/6 trees)."""
    tiles = -(-rows // 512)
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
    f64, ops + * / - cos exp, 20 populations, default options), lock-step islands with one batched
    device scoring call per evolution round (sr_amd.search.equation_search).  Iterations/sec counts
    completed s_r_cycles (one per island per iteration, src/SymbolicRegression.jl:1091) per wall s."""
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
            "config": "C1 README example, X=randn(2,100) f64, 20 populations, default options"}


PROFILED_STEPS = 6  # steps + warmup of the bench command tools/profile.sh profiles


def measured_traffic():
    """Per-launch HBM bytes of the interpreter kernel from the committed rocprofv3 PMC pass of this
    same command (profiles/traffic.json, written by tools/profile.sh: FETCH_SIZE x2, gfx950)."""
    p = os.path.join(ROOT, "profiles", "traffic.json")
    try:
        with open(p) as f:
            t = json.load(f)
    except (OSError, ValueError):
        return None
    # per step: every interpreter launch of the profiled run (chunks and dead-tree probes) over its
    # steps (tools/profile.sh runs bench.py --steps 5 --warmup 1)
    t["hbm_read_bytes_per_step"] = t["hbm_read_bytes_per_launch"] * t["calls"] / PROFILED_STEPS
    t["source"] = "profiles/traffic.json (rocprofv3 --pmc FETCH_SIZE of bench.py)"
    return t


def cpu_baseline(opts, tb, X, y, n_sample):
    """Oracle (C port of DE's array-at-a-time evaluator, OpenMP over trees) on a bounded sample:
    a strided subset of the same trees over all rows (~10-30 s on 16 host cores)."""
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
        "sample": f"{sub.n_trees} of {tb.n_trees} trees (every {step}th), all {X.shape[1]} rows, {dt:.1f} s",
    }


if __name__ == "__main__":
    main()
