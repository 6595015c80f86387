"""CPU, world_size 2 (gloo): island-sharded equation_search (SURVEY §8(e) island sharding).

Two processes each own half of the islands (island i on rank i % 2), score only their islands'
children, all-gather the islands after every iteration and replay the head node's bookkeeping
(statistics, hall of fame, Pareto frontier, migration by the owner).  The scorer is the oracle
(CPU test stand-in for the device call, injected through ``_loss_fn``); the search engine and the
exchange are the product code.  Random streams and birth counters are per island, so the sharded
search must reproduce the single-process search exactly: same hall of fame, same populations.
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


def _setup(batching=False):
    sys.path[:0] = [os.path.join(ROOT, "symbolicregression.jl_amd"), os.path.join(ROOT, "oracle")]
    from oracle import Oracle
    from sr_amd import Options

    opts = Options(binary_operators=["+", "*", "/", "-"], unary_operators=["cos", "exp"], populations=4,
                   population_size=12, ncycles_per_iteration=25, maxsize=15, should_optimize_constants=False,
                   batching=batching, batch_size=30)
    rng = np.random.default_rng(0)
    X = rng.standard_normal((2, 100))
    y = 2 * np.cos(X[1]) + X[0] ** 2 - 2
    orc = Oracle.from_options(opts)

    def score(tb, rows):
        Xv, yv = (X, y) if rows is None else (X[:, rows], y[rows])
        losses, comp = orc.eval_loss_batch(tb, Xv, yv, accum="ref")
        return np.where(comp, losses, np.inf)

    return opts, X, y, score


def _summary(res):
    from sr_amd import string_tree

    hof = [(m.complexity, m.cost, m.loss, string_tree(m.tree)) for m, e in zip(res.hall_of_fame.members,
                                                                          res.hall_of_fame.exists) if e]
    pops = [[(m.cost, m.birth, string_tree(m.tree)) for m in p] for p in res.populations]
    return hof, pops


def _worker(rank, world, port, q, batching):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    opts, X, y, score = _setup(batching)
    from sr_amd import equation_search

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        res = equation_search(X, y, niterations=3, options=opts, seed=5, distributed=True, _loss_fn=score)
        q.put((rank, _summary(res), res.num_evals))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("batching", [False, True])
def test_island_sharded_search_equals_single_process(batching):
    """(batching: one minibatch per iteration from a stream keyed by (seed, iteration), the same on
    every rank, so the sharded search still equals the single-process one.)"""
    import torch.multiprocessing as mp

    opts, X, y, score = _setup(batching)
    from sr_amd import equation_search

    single = equation_search(X, y, niterations=3, options=opts, seed=5, _loss_fn=score)
    ref = _summary(single)

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q, batching)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(2)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort(key=lambda r: r[0])
    for rank, summ, num_evals in res:
        assert summ[0] == ref[0], f"rank {rank}: hall of fame differs"
        assert summ[1] == ref[1], f"rank {rank}: populations differ"
        assert num_evals == pytest.approx(single.num_evals, rel=1e-12)  # (fractional evals summed per rank)
    # the search made progress: something beats the best constant (the size-1 entry) clearly
    assert len(ref[0]) > 3 and min(h[2] for h in ref[0]) < 0.8 * ref[0][0][2]
