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


def test_ddp_two_ranks_identical_parameters():
    env = dict(os.environ, RPC_DIST_BACKEND="gloo", HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), os.path.join(ROOT, "tools", "ddp_check.py")]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-3000:]
    assert '"ddp": "ok"' in out, out[-3000:]
