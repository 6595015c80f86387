"""GPU, RCCL: row sharding and tree sharding through the library's own RCCL
communicator (C ABI sr_comm_*; torch.distributed's gloo group only broadcasts the unique id).

One process, world size 1, on device 0 (a box has one GPU; RCCL refuses two ranks on one device):
`sr_eval_loss_sharded` (the whole row-sharded step: packed partials + error word through ONE
in-place ncclAllReduce, device finalize, the exact Julia-order pass for BIG trees) and
`sr_eval_loss_tree_sharded` must equal the single-GPU `eval_loss_batch` (flags bit for bit, losses to
1e-6) and the oracle's flags.  torch never touches the GPU here: its bundled HIP runtime cannot share
the device with the library's (measured on the box: whichever initialises second sees no GPU).  The
multi-rank protocols are covered on CPU by tests/test_distributed.py (gloo, world size 2).
"""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from sr_amd import Dataset, Options, eval_loss_batch, flatten_trees, gen_random_population, parse_expression

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _population(n=1 << 17, seed=5):
    rng = np.random.default_rng(seed)
    X = rng.standard_normal((5, n)).astype(np.float32)
    X[2, :3000] = np.float32(2e35)  # big finite values: trees over x3 take the exact (BIG) path
    y = (2 * np.cos(X[3]) + X[0] ** 2 - 2).astype(np.float32)
    opts = Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp", "log"])
    trees = gen_random_population(2000, opts, 5, seed=8)
    trees += [parse_expression(e, opts) for e in ("x3 * 1.0", "x3 + x1", "(x3 * 0.5) - x2", "cos(x1) * x2")]
    return X, y, opts, flatten_trees(trees, np.float32)


def test_sharded_rccl_world1_matches_single_gpu():
    import torch.distributed as dist

    import sr_amd
    from oracle import Oracle
    from sr_amd.distributed import (comm_info, destroy_device_comm, eval_loss_sharded, eval_loss_tree_sharded,
                                    gpu_partials_allreduce, init_device_comm)

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1)
    ctx = sr_amd.get_context()
    try:
        init_device_comm(ctx=ctx)
        assert ctx.has_comm
        info = comm_info(ctx)
        assert (info["nranks"], info["rank"]) == (1, 0)
        assert os.path.dirname(info["hip"]) == os.path.dirname(info["rccl"]), info
        X, y, opts, tb = _population()
        n = X.shape[1]
        ds = Dataset(X, y)

        packed = gpu_partials_allreduce(tb, ds, opts, n)
        assert packed.shape == (5, tb.n_trees)
        assert np.any(packed[2] > 0), "no tree took the BIG (exact-sum) path"

        ref_loss, ref_comp = eval_loss_batch(tb, ds, opts)
        _, oc = Oracle.from_options(opts).eval_loss_batch(tb, X, y, n_threads=8)
        assert np.array_equal(ref_comp, oc)
        sel = ref_comp & np.isfinite(ref_loss)
        for name, (loss, comp) in (("rows", eval_loss_sharded(tb, ds, opts, n)),
                                   ("trees", eval_loss_tree_sharded(tb, ds, opts))):
            assert np.array_equal(comp, ref_comp), name
            assert 0.1 < comp.mean() < 0.9
            rel = np.abs(loss[sel].astype(np.float64) - ref_loss[sel]) / np.maximum(np.abs(ref_loss[sel]), 1e-30)
            assert float(rel.max(initial=0.0)) < 1e-6, name
            assert np.all(np.isinf(loss[~comp])), name
        # on data without huge values the row-sharded step uses the single-GPU launch pipeline, derived
        # columns included (every rank decides them from all shards' statistics)
        Xc, yc = X.copy(), y.copy()
        Xc[2, :3000] = 0.5
        dsc = Dataset(Xc, yc)
        loss, comp = eval_loss_sharded(tb, dsc, opts)
        assert ctx.last_derived_columns() > 0
        ref_loss, ref_comp = eval_loss_batch(tb, dsc, opts)
        assert np.array_equal(comp, ref_comp)
        sel = ref_comp & np.isfinite(ref_loss)
        assert np.array_equal(loss[sel], ref_loss[sel])  # the same launches: bit-identical
    finally:
        destroy_device_comm(ctx)
        dist.destroy_process_group()


_ORDER_SCRIPT = r"""
import json, os, socket, sys
sys.path[:0] = [os.path.join(ROOT, "symbolicregression.jl_amd"), os.path.join(ROOT, "tests")]
import torch.distributed as dist          # torch's bundled ROCm is loaded BEFORE the library
import numpy as np
import sr_amd
from sr_amd.distributed import comm_info, eval_loss_sharded, init_device_comm
from test_gpu_rccl import _population
with socket.socket() as s:
    s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]
dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
ctx = sr_amd.get_context()
init_device_comm(ctx=ctx)
X, y, opts, tb = _population(1 << 16, seed=6)
ds = sr_amd.Dataset(X, y)
loss, comp = eval_loss_sharded(tb, ds, opts)
ref, rcomp = sr_amd.eval_loss_batch(tb, ds, opts)
sel = rcomp & np.isfinite(ref)
print(json.dumps(dict(comm_info(ctx), same=bool(np.array_equal(comp, rcomp)),
                      maxrel=float(np.max(np.abs(loss[sel] - ref[sel]) / np.abs(ref[sel]), initial=0.0)))))
dist.destroy_process_group()
"""


def test_import_order_torch_first_keeps_one_runtime():
    """A process that imports torch.distributed before sr_amd (a user script, Julia via PyCall): the
    loader then binds the library to torch's already-loaded HIP runtime and RCCL (same sonames), and the
    library's check keeps HIP and RCCL from ONE tree; the sharded step still equals the single call."""
    import json

    code = "ROOT = %r\n" % ROOT + _ORDER_SCRIPT
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-3000:]
    info = json.loads(out.stdout.strip().splitlines()[-1])
    print(info)
    assert os.path.dirname(info["hip"]) == os.path.dirname(info["rccl"]), info
    assert info["same"] and info["maxrel"] < 1e-6, info
