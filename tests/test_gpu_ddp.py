"""(e) the data-parallel step on the GPU: two ranks under torch.distributed.run (gloo, sharing the one
GPU of the test box) train the real KITTI model for 3 steps under DDP; parameters must stay
bit-identical across ranks (tools/ddp_check.py). The 8-GPU bench runs the same code over nccl (RCCL)."""
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(nproc, backend=None, classes=3):
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", RPC_DDP_CLASSES=str(classes))
    env.pop("RPC_DIST_BACKEND", None)
    if backend:
        env["RPC_DIST_BACKEND"] = backend
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(nproc),
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), os.path.join(ROOT, "tools", "ddp_check.py")]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-3000:]
    assert '"ddp": "ok"' in out, out[-3000:]
    if nproc > 1:
        assert '"averaged_grads_ok": true' in out, out[-3000:]
    print(out[-600:])
    return out


def test_ddp_two_ranks_identical_parameters():
    """Two ranks share the box's one GPU over gloo (RCCL refuses two ranks on one device)."""
    _run(2, backend="gloo", classes=3)


def test_ddp_rccl_backend_one_rank():
    """The RCCL path: backend nccl (= RCCL on ROCm), DDP's bucketed all-reduce and an explicit
    all_reduce through the RCCL communicator, 3-class model (the 8xb6 config's per-rank step)."""
    out = _run(1, backend=None, classes=3)
    assert '"backend": "nccl"' in out, out[-3000:]
    assert '"all_reduce_ok": true' in out, out[-3000:]


def test_bench_gpus2_spawns_two_ranks():
    """bench.py --gpus 2 from a plain `python` starts torch.distributed.run with two ranks (gloo so
    both share the test box's one GPU) and reports n_gpus = the process-group world size."""
    import json
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", RPC_DIST_BACKEND="gloo")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--no-cpu-baseline"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-3000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("{")][-1]
    res = json.loads(line)
    assert res["n_gpus"] == 2 and res["config"]["parallelism"] == "dp2", res
    assert "3-class" in res["config"]["workload"], res
    assert res["config"]["dist_backend"] == "gloo"
