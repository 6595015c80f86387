"""GPU, RCCL: the row-sharded combine through the library's own RCCL communicator
(C ABI sr_comm_*; torch.distributed's gloo group only broadcasts the unique id).

One process, world size 1, on device 0 (a box has one GPU; RCCL refuses two ranks on one device):
the packed [4, n_trees] partials are summed by ONE in-place ncclAllReduce on the device
(`sr_eval_loss_partials_allreduce`), the BIG trees go through the per-shard Julia-order folds +
`sr_jsum_finite`, and `sr_finalize_losses` finishes.  The result must equal the single-GPU
`eval_loss_batch` (flags bit for bit, losses to 1e-6) and the oracle's flags.  torch never touches
the GPU here: its bundled HIP runtime cannot share the device with the library's (measured on the
box: whichever initialises second sees no GPU).  The two-rank combine is covered on CPU by
tests/test_distributed.py (gloo).
"""
import socket

import numpy as np
import pytest

from sr_amd import Dataset, Options, eval_loss_batch, flatten_trees, gen_random_population, parse_expression

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_row_sharded_rccl_world1_matches_single_gpu():
    import torch.distributed as dist

    import sr_amd
    from oracle import Oracle
    from sr_amd.distributed import eval_loss_sharded, gpu_partials_allreduce, init_device_comm

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1)
    ctx = sr_amd.get_context()
    try:
        init_device_comm(ctx=ctx)
        assert ctx.has_comm
        rng = np.random.default_rng(5)
        n = 1 << 17
        X = rng.standard_normal((5, n)).astype(np.float32)
        X[2, :3000] = np.float32(2e35)  # big finite values: trees over x3 take the exact (BIG) path
        y = (2 * np.cos(X[3]) + X[0] ** 2 - 2).astype(np.float32)
        opts = Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp", "log"])
        trees = gen_random_population(2000, opts, 5, seed=8)
        trees += [parse_expression(e, opts) for e in ("x3 * 1.0", "x3 + x1", "(x3 * 0.5) - x2", "cos(x1) * x2")]
        tb = flatten_trees(trees, np.float32)
        ds = Dataset(X, y)

        packed = gpu_partials_allreduce(tb, ds, opts, n)
        assert packed.shape == (4, tb.n_trees)
        assert np.any(packed[2] > 0), "no tree took the BIG (exact-sum) path"

        loss, comp = eval_loss_sharded(tb, ds, opts, n)
        ref_loss, ref_comp = eval_loss_batch(tb, ds, opts)
        assert np.array_equal(comp, ref_comp)
        assert 0.1 < comp.mean() < 0.9
        sel = ref_comp & np.isfinite(ref_loss)
        rel = np.abs(loss[sel].astype(np.float64) - ref_loss[sel]) / np.maximum(np.abs(ref_loss[sel]), 1e-30)
        assert float(rel.max(initial=0.0)) < 1e-6
        _, oc = Oracle.from_options(opts).eval_loss_batch(tb, X, y, n_threads=8)
        assert np.array_equal(comp, oc)
    finally:
        from sr_amd import _lib

        _lib.check(_lib.lib.sr_comm_destroy(ctx.handle))
        ctx.has_comm = False
        dist.destroy_process_group()
