"""CPU: bench.py's own rank launcher (`--gpus N` without torchrun) and CPU channel, rehearsed with
--dry-run (no device): N fresh rank processes rendezvous over gloo, time between barriers, take the
max over ranks, and rank 0 prints one JSON line with n_gpus = N.  The same under
torch.distributed.run (the driver's multi-GPU launcher)."""
import json
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _last_json(out):
    return json.loads([ln for ln in out.splitlines() if ln.startswith("{")][-1])


def test_bench_spawns_its_own_ranks():
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run", "--steps", "3",
                          "--warmup", "1"], capture_output=True, text=True, timeout=240,
                         env={k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")})
    assert out.returncode == 0, out.stderr[-2000:]
    line = _last_json(out.stdout)
    assert line["n_gpus"] == 2 and line["ranks_launched_by"] == "bench.py"
    assert line["ms_per_step"] >= 2.0  # the max over ranks (rank 1 sleeps 2 ms per step)


def test_bench_under_torchrun():
    out = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                          "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"),
                          "--gpus", "2", "--dry-run", "--steps", "3", "--warmup", "1"],
                         capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-2000:]
    line = _last_json(out.stdout)
    assert line["n_gpus"] == 2 and line["ranks_launched_by"] == "launcher"
