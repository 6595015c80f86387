"""GPU, two ranks on one device: the library's OWN multi-rank code.

`sr_eval_loss_sharded` and `sr_eval_loss_tree_sharded` run with nranks = 2 in two processes on GPU 0,
their collectives going through `sr_comm_init_host` (the caller's gloo group instead of RCCL, which
refuses two ranks on one device).  Everything else is the C++ path the 8-GPU run takes: the shard
layout exchange, the packed all-reduce with its error word, the exact Julia-order pass whose leaf
blocks straddle the cut between the shards (head ranges), every complete tree's in-order loss fold
walked rank after rank (round 6), the tree owners' results all-gather, and the failure protocol (an
injected buffer failure on one rank makes BOTH ranks return an error; so does an injected HIP failure
on one rank after the packed all-reduce, after the exact pass's all-gather, in the loss folds'
gathers, or in the weights' sum gather of a weighted call; the next call works on both).

Uneven shards (rank 0 holds 60,001 of 143,417 rows), huge values around the cut (BIG trees), weights.
Results must equal the single-GPU call on the whole dataset (flags and losses bit for bit: both are the
in-order fold) and the oracle's flags.
"""
import os
import socket
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N_TOTAL = (1 << 17) + 12345
CUT = 60001
M = 3.4028235677973366e38


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _data(weighted):
    rng = np.random.default_rng(21)
    X = rng.standard_normal((5, N_TOTAL)).astype(np.float32)
    X[2, CUT - 700:CUT + 900] = np.float32(2e35)  # BIG trees over x3; their leaf blocks straddle the cut
    y = (2 * np.cos(X[3]) + X[0] ** 2 - 2).astype(np.float32)
    w = (0.5 + rng.random(N_TOTAL)).astype(np.float32) if weighted else None
    return X, y, w


def _trees(opts):
    from sr_amd import flatten_trees, gen_random_population, parse_expression

    trees = gen_random_population(1500, opts, 5, seed=31)
    trees += [parse_expression(e, opts) for e in ("x3 * 1.0", "x3 + x1", "(x3 * 0.5) - x2", "cos(x1) * x2")]
    # the loss fold near overflow: Σ (c x1)^2 within +-0.5 % of the threshold (folded in row order, the
    # fold continued from rank 0's shard into rank 1's)
    X, _, _ = _data(False)
    s2 = float(np.sum(X[0].astype(np.float64) ** 2))
    trees += [parse_expression(f"x1 * {float(np.float32(np.sqrt(M * f / s2)))!r}", opts) for f in (0.996, 0.9995, 1.0005, 1.004)]
    return flatten_trees(trees, np.float32)


def _worker(rank, world, port, q):
    sys.path[:0] = [os.path.join(ROOT, "symbolicregression.jl_amd"), os.path.join(ROOT, "tests"),
                    os.path.join(ROOT, "oracle")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), SR_AMD_DEVICE="0")
    import torch.distributed as dist

    import sr_amd
    from sr_amd import Dataset, Options, eval_loss_batch
    from sr_amd.distributed import comm_info, eval_loss_sharded, eval_loss_tree_sharded, init_host_comm

    dist.init_process_group("gloo", rank=rank, world_size=world)
    out = {"rank": rank}
    try:
        ctx = sr_amd.get_context()
        init_host_comm(ctx=ctx)
        info = comm_info(ctx)
        out["comm"] = (info["nranks"], info["rank"], info["transport"])
        opts = Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp", "log"])
        tb = _trees(opts)
        lo, hi = (0, CUT) if rank == 0 else (CUT, N_TOTAL)
        for weighted in (False, True):
            X, y, w = _data(weighted)
            shard = Dataset(np.ascontiguousarray(X[:, lo:hi]), np.ascontiguousarray(y[lo:hi]),
                            weights=None if w is None else np.ascontiguousarray(w[lo:hi]))
            full = Dataset(X, y, weights=w)
            ref_loss, ref_comp = eval_loss_batch(tb, full, opts)
            ref_fold = ctx.last_fold_trees()
            loss, comp = eval_loss_sharded(tb, shard, opts)
            key = "w" if weighted else "u"
            out[key + "_rows"] = (loss, comp, ctx.last_exact_trees(), ctx.last_fold_trees())
            out[key + "_ref"] = (ref_loss, ref_comp, ref_fold)
            tl, tc = eval_loss_tree_sharded(tb, full, opts)
            out[key + "_trees"] = (tl, tc)
        # the failure protocol: a fresh communicator starts with empty collective buffers, so the next
        # call grows them on both ranks; rank 1's growth is made to fail -> both ranks raise, and the
        # next call works on both
        X, y, _ = _data(False)
        shard = Dataset(np.ascontiguousarray(X[:, lo:hi]), np.ascontiguousarray(y[lo:hi]))
        big = tb.take(np.concatenate([np.arange(tb.n_trees)] * 3))
        errs = []
        for fn in (lambda: eval_loss_sharded(big, shard, opts), lambda: eval_loss_tree_sharded(big, Dataset(X, y), opts)):
            init_host_comm(ctx=ctx)
            if rank == 1:
                ctx.set_tuning("inject_failure", 1)
            try:
                fn()
                errs.append(None)
            except Exception as e:  # noqa: BLE001
                errs.append(str(e)[:200])
            ctx.set_tuning("inject_failure", 0)
        out["errors"] = errs
        out["after"] = eval_loss_sharded(big, shard, opts)
        # local HIP failures AFTER a collective: after the packed all-reduce, after
        # the exact pass's all-gather, and in the loss fold's gathers (the first, and the last of the
        # chain, which only the final agreement catches); the band and BIG trees make every later
        # collective run, so a rank returning alone would leave its peer waiting
        post = []
        # (a weighted call's Base.sum(w) gather: ADVICE r5, a failure there must fail both ranks too)
        Xw, yw, ww = _data(True)
        wshard = Dataset(np.ascontiguousarray(Xw[:, lo:hi]), np.ascontiguousarray(yw[lo:hi]),
                         weights=np.ascontiguousarray(ww[lo:hi]))
        for knob, who, k, ds_ in (("inject_failure_post", 1, 1, shard), ("inject_failure_post_exact", 0, 1, shard),
                                  ("inject_failure_post_gather", 1, 1, shard), ("inject_failure_post_gather", 0, 3, shard),
                                  ("inject_failure_post_gather", 1, 5, shard), ("inject_failure_post_wsum", 0, 1, wshard)):
            if rank == who:
                ctx.set_tuning(knob, k)
            try:
                eval_loss_sharded(tb, ds_, opts)
                post.append(None)
            except Exception as e:  # noqa: BLE001
                post.append(str(e)[:200])
            ctx.set_tuning(knob, 0)
        out["post_errors"] = post
        out["post_after"] = eval_loss_sharded(tb, shard, opts)
        q.put(out)
    except Exception as e:  # noqa: BLE001
        import traceback

        out["fatal"] = traceback.format_exc()[-3000:]
        q.put(out)
    finally:
        dist.destroy_process_group()


def test_two_ranks_on_one_gpu_run_the_library_sharded_paths():
    import torch.multiprocessing as mp

    from oracle import Oracle
    from sr_amd import Options

    mpc = mp.get_context("spawn")
    q = mpc.Queue()
    port = _free_port()
    procs = [mpc.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = sorted((q.get(timeout=400) for _ in range(2)), key=lambda d: d["rank"])
    for p in procs:
        p.join(timeout=60)
    for g in got:
        assert "fatal" not in g, g.get("fatal")
    assert [g["comm"] for g in got] == [(2, 0, "host"), (2, 1, "host")]
    opts = Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp", "log"])
    tb = _trees(opts)
    orc = Oracle.from_options(opts)
    for key in ("u", "w"):
        X, y, w = _data(key == "w")
        _, o_comp = orc.eval_loss_batch(tb, X, y, w, n_threads=8)
        ref_loss, ref_comp, ref_fold = got[0][key + "_ref"]
        assert np.array_equal(ref_comp, o_comp), key
        assert ref_fold > 0, "no tree took the in-order fold"
        for g in got:
            loss, comp, n_exact, n_fold = g[key + "_rows"]
            assert n_exact > 0, (key, "no tree took the exact (BIG) pass")
            assert n_fold >= 1, (key, n_fold, ref_fold)  # (the band trees, and any walk that fell back)
            assert np.array_equal(comp, ref_comp), key
            assert np.array_equal(np.isinf(loss), np.isinf(ref_loss)), key
            # every complete tree's loss is the in-order fold across the two shards (round 6): the single
            # call's bits (NaN losses compare as NaN)
            sel = comp & ~np.isnan(ref_loss)
            assert np.array_equal(loss[sel].view(np.uint32), ref_loss[sel].view(np.uint32)), key
            # the band trees (the last four) are folded in row order across the shards: bit for bit
            assert np.array_equal(loss[-4:].view(np.uint32), ref_loss[-4:].view(np.uint32)), (key, loss[-4:], ref_loss[-4:])
            tl, tc = g[key + "_trees"]
            assert np.array_equal(tc, ref_comp), key
            assert np.array_equal(tl.view(np.uint32), ref_loss.view(np.uint32)), key  # the same single-GPU calls
        assert 0.1 < ref_comp.mean() < 0.9
    for g in got:
        assert all(e is not None for e in g["errors"]), g["errors"]  # both ranks failed, neither hung
        loss, comp = g["after"]
        assert np.array_equal(comp, np.concatenate([got[0]["u_ref"][1]] * 3))
        assert all(e is not None for e in g["post_errors"]), g["post_errors"]  # failures after a collective
        loss, comp = g["post_after"]
        assert np.array_equal(comp, got[0]["u_ref"][1])
