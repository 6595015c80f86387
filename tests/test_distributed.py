"""CPU, world_size 2 (gloo): the multi-GPU protocols of row sharding and tree sharding.

`sr_amd.distributed.eval_loss_sharded` is run by two processes over two row shards with CPU
stand-ins for the two GPU calls (per-shard packed partials — Σ loss + flag bits — from the oracle's
predictions, and per-shard Julia-order folds of the checked arrays); the single packed all-reduce,
the BIG-tree exact path (all-gather + `sr_jsum_finite`) and `sr_finalize_losses` (host C ABI) are
the product code.  The result must equal the oracle on the unsharded data.  Tree sharding deals the
trees over the ranks (`tree_owners`, the library's rule) and one all-reduce hands every rank every
result.  A failure on one rank is all-reduced as an error word: every rank raises, none hangs.
"""
import os
import socket
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _data():
    rng = np.random.default_rng(0)
    n = 4000
    X = rng.standard_normal((3, n)).astype(np.float32)
    X[0] = np.abs(X[0]) + 1.0  # keeps x1 * 1e35 finite per row
    y = (np.cos(X[1]) + X[2]).astype(np.float32)
    return X, y


EXPRS = ["cos(x2) + x3", "x2 * x3 - 1.5", "log(x2)", "x1 * 1e35", "x1 * 1e34", "cos(x1) * x2 / x3"]


def _worker(rank, world, port, q, mode="rows"):
    sys.path[:0] = [os.path.join(ROOT, "symbolicregression.jl_amd"), os.path.join(ROOT, "oracle")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    from oracle import Oracle
    from sr_amd import Dataset, Options, flatten_trees, parse_expression
    from sr_amd import _lib
    from sr_amd.distributed import eval_loss_sharded, jsum_ranges
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from test_jsum import jl_sum

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        X, y = _data()
        n = X.shape[1]
        lo, hi = rank * n // world, (rank + 1) * n // world
        Xs, ys = np.ascontiguousarray(X[:, lo:hi]), np.ascontiguousarray(y[lo:hi])
        shard = Dataset(Xs, ys)
        opts = Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "log"])
        tb = flatten_trees([parse_expression(e, opts) for e in EXPRS], np.float32)
        orc = Oracle.from_options(opts)
        tbig = np.float32(3.4028235e38 / (2.0 * n))

        def partials(tb_):
            packed = np.zeros((5, tb_.n_trees))
            for k in range(tb_.n_trees):
                out, _ = orc.eval_tree_array(tb_, k, Xs)
                if not np.all(np.isfinite(out)):
                    packed[1, k] = 1.0  # SR_FLAG_NONFINITE
                elif np.any(np.abs(out) >= tbig):
                    packed[2, k] = 1.0  # SR_FLAG_BIG
                packed[0, k] = np.sum((out.astype(np.float64) - ys) ** 2)
            return packed

        def exact(tb_, lst, max_checks, row_offset):
            # these trees' only checked array is the root: its Julia-order folds over this shard's ranges
            lo_, hi_, _, _ = jsum_ranges(row_offset, Xs.shape[1], n)
            out = np.zeros((len(lst), 1, len(lo_)), dtype=np.float32)
            for i, k in enumerate(lst):
                a = orc.eval_tree_array(tb_, int(k), Xs)[0].astype(np.float32)
                out[i, 0] = [jl_sum(a, int(l), int(h)) for l, h in zip(lo_, hi_)]
            return out

        if mode == "rows":
            loss, comp = eval_loss_sharded(tb, shard, opts, n, partials_fn=partials, exact_fn=exact)
        elif mode == "trees":
            from sr_amd.distributed import eval_loss_tree_sharded

            # replicated dataset; this rank scores only its share (the oracle stands in for the GPU)
            def score(sub):
                assert sub.n_trees < tb.n_trees
                return orc.eval_loss_batch(sub, X, y, accum="f64")
            loss, comp = eval_loss_tree_sharded(tb, Dataset(X, y), opts, score_fn=score)
        else:  # "fail": rank 1's GPU call fails; both ranks must raise instead of waiting for each other
            def failing(tb_):
                if rank == 1:
                    raise RuntimeError("injected failure")
                return partials(tb_)
            try:
                eval_loss_sharded(tb, shard, opts, n, partials_fn=failing, exact_fn=exact)
                q.put((rank, "no error", None))
            except RuntimeError as e:
                q.put((rank, str(e), None))
            return
        q.put((rank, loss.tolist(), comp.tolist()))
    finally:
        dist.destroy_process_group()


def _run(mode):
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q, mode)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(2)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort()
    return res


@pytest.mark.parametrize("mode", ["rows", "trees"])
def test_sharded_combine_gloo_world2(mode):
    sys.path[:0] = [os.path.join(ROOT, "symbolicregression.jl_amd"), os.path.join(ROOT, "oracle")]
    from oracle import Oracle
    from sr_amd import Options, flatten_trees, parse_expression

    res = _run(mode)
    assert res[0][1:] == res[1][1:]  # every rank finalizes the same answer
    loss, comp = np.array(res[0][1], dtype=np.float32), np.array(res[0][2])

    X, y = _data()
    opts = Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "log"])
    tb = flatten_trees([parse_expression(e, opts) for e in EXPRS], np.float32)
    ol, oc = Oracle.from_options(opts).eval_loss_batch(tb, X, y, accum="f64")  # (the Python protocol combines f64 partials)
    # x1*1e35 / x1*1e34: rows are finite and big; only the exact global array sum decides (BIG path)
    assert list(comp) == list(oc) == [True, True, False, False, True, True]
    for k in np.nonzero(oc)[0]:
        if np.isfinite(ol[k]):
            assert loss[k] == pytest.approx(float(ol[k]), rel=1e-6), EXPRS[k]
        else:
            assert np.isinf(loss[k])


def test_failure_on_one_rank_fails_every_rank():
    res = _run("fail")
    assert res[0][1] == "the row-sharded step failed on a peer rank"
    assert res[1][1] == "injected failure"


def test_tree_owners_balanced():
    sys.path[:0] = [os.path.join(ROOT, "symbolicregression.jl_amd")]
    from sr_amd import Options, flatten_trees, gen_random_population
    from sr_amd.distributed import tree_owners

    opts = Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp", "log"])
    tb = flatten_trees(gen_random_population(10_000, opts, 5, seed=1), np.float32)
    sizes = np.diff(tb.offsets)
    for world in (1, 2, 3, 8):
        own = tree_owners(tb, world)
        assert set(own.tolist()) == set(range(world))
        load = np.array([sizes[own == r].sum() for r in range(world)])
        assert load.max() - load.min() <= sizes.max(), (world, load)
