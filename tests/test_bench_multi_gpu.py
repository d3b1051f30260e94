"""Rehearsal of the driver's multi-GPU bench command on the one-GPU box.

The driver runs ``python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N`` on an
8-GPU node at round end; this runs the same code path with 2 ranks that share the box's GPU
(``STF_DIST_BACKEND=gloo``: RCCL needs one GPU per rank), once through bench.py's own launcher
(``--gpus 2`` without WORLD_SIZE starts the ranks as a child torch.distributed.run) and once through
an explicit torch.distributed.run, for the default workload (configs[1], UNet) and configs[3]'s per-GPU
STF workload (--config 4).  The JSON line must be the N=2 line: n_gpus 2, parallelism dp2, the
global batch twice the per-GPU batch, weak scaling, and no N=1-only legs (dice, CPU baseline)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(args, launcher):
    env = dict(os.environ, STF_DIST_BACKEND="gloo")
    env.pop("WORLD_SIZE", None)
    if launcher:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
               "--master-addr", "127.0.0.1", f"--master-port={_free_port()}", "bench.py", "--gpus", "2"] + args
    else:
        cmd = [sys.executable, "bench.py", "--gpus", "2"] + args
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, (r.returncode, r.stdout[-2000:], r.stderr[-4000:])
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]           # rank 0 alone prints
    return json.loads(lines[0])


@pytest.mark.parametrize("args,launcher,per_gpu", [
    (["--steps", "2", "--warmup", "2"], False, 64),
    (["--config", "4", "--steps", "2", "--warmup", "2"], True, 16),
])
def test_bench_two_ranks_on_one_gpu(args, launcher, per_gpu):
    d = _run(args, launcher)
    c = d["config"]
    assert d["n_gpus"] == 2 and c["parallelism"] == "dp2" and d["scaling"] == "weak"
    assert c["per_gpu_batch"] == per_gpu and c["global_batch"] == 2 * per_gpu
    assert d["steps"] == 2 and d["value"] > 0 and d["ms_per_step"] > 0
    assert abs(d["value"] - 2 * per_gpu * 1e3 / d["ms_per_step"]) <= 1e-3 * d["value"]
    assert "dice_vs_ref" not in d and "cpu_baseline" not in d
    assert d["execution"] == "native_plan"
