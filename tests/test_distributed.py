"""CPU, world_size 2 (gloo): the multi-GPU combine of row-sharded partials.

`sr_amd.distributed.eval_loss_sharded` is run by two processes over two row shards with CPU
stand-ins for the two GPU calls (per-shard packed partials — Σ loss + flag bits — from the oracle's
predictions, and per-shard Julia-order folds of the checked arrays); the single packed all-reduce,
the BIG-tree exact path (all-gather + `sr_jsum_finite`) and `sr_finalize_losses` (host C ABI) are
the product code.  The result must equal the oracle on the unsharded data.
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


def _worker(rank, world, port, q):
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
            packed = np.zeros((4, tb_.n_trees))
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

        loss, comp = eval_loss_sharded(tb, shard, opts, n, partials_fn=partials, exact_fn=exact)
        q.put((rank, loss.tolist(), comp.tolist()))
    finally:
        dist.destroy_process_group()


def test_sharded_combine_gloo_world2():
    import torch.multiprocessing as mp

    sys.path[:0] = [os.path.join(ROOT, "symbolicregression.jl_amd"), os.path.join(ROOT, "oracle")]
    from oracle import Oracle
    from sr_amd import Options, flatten_trees, parse_expression

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(2)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort()
    assert res[0][1:] == res[1][1:]  # every rank finalizes the same answer
    loss, comp = np.array(res[0][1], dtype=np.float32), np.array(res[0][2])

    X, y = _data()
    opts = Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "log"])
    tb = flatten_trees([parse_expression(e, opts) for e in EXPRS], np.float32)
    ol, oc = Oracle.from_options(opts).eval_loss_batch(tb, X, y)
    # x1*1e35 / x1*1e34: rows are finite and big; only the exact global array sum decides (BIG path)
    assert list(comp) == list(oc) == [True, True, False, False, True, True]
    for k in np.nonzero(oc)[0]:
        if np.isfinite(ol[k]):
            assert loss[k] == pytest.approx(float(ol[k]), rel=1e-6), EXPRS[k]
        else:
            assert np.isinf(loss[k])
