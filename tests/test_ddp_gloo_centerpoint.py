"""(e) multi-GPU path on CPU for config 4's detector: world_size-2 `gloo` run of Trainer.step_batch under
DDP with the plugin AdversarialCenterPoint (models/detectors/adversarial_centerpoint.py:43-257).

Same construction as tests/test_ddp_gloo.py: each rank takes one frame of the golden `centerpoint_e3`
fixture (stand-in VFE / middle / CenterHead, CPU oracle perturber with its tensors as parameters in the
adversary slot) and one optimizer step. The result must equal a single-process reference that averages the
two per-shard gradients, clips them to 0.5 and takes the same AdamW step (adversary lr_mult 2.0), and both
ranks must hold identical parameters. The per-rank parts CenterPoint adds over VoxelNet — the detection
total clamped to [0, 100] before the adaptive adversarial weight, the l2 term from the perturber's own
norm — are computed on each rank's shard, as DDP runs the reference.
"""
import os

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
from torch import nn

from robustpointclouds_amd.adversarial_loss import parse_losses
from robustpointclouds_amd.trainer import Trainer
from tests.test_adversarial_centerpoint import OracleAdversary, StandInVFE5, _load, _model, _Sample
from tests.test_ddp_gloo import _free_port

WORLD = 2
TAG = "e3"


class ParamOracleAdversary(OracleAdversary):
    """The oracle perturber with its tensors registered as parameters (so DDP / AdamW see them)."""

    def __init__(self, d, hidden):
        super().__init__(d, hidden)
        self.params = nn.ParameterDict({k: nn.Parameter(v.detach().clone()) for k, v in self.op.p.items()})
        self.op.p = dict(self.params.items())


def _build(d):
    torch.manual_seed(0)
    m = _model(d, StandInVFE5(), torch.device("cpu"))
    m.adversary = ParamOracleAdversary(d, [int(h) for h in d["hidden"]])
    return m


def _shard(d, r):
    sel = d["coors"][:, 0] == r
    coors = d["coors"][sel].copy()
    coors[:, 0] = 0
    return {"voxels": {"voxels": torch.from_numpy(d["vox"][sel]),
                       "num_points": torch.from_numpy(d["num_points"][sel]),
                       "coors": torch.from_numpy(coors)}, "batch_size": 1}


def _worker(rank, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        d = _load(TAG)
        m = _build(d)
        tr = Trainer(m, lr=1e-2, ddp=True, device=torch.device("cpu"), iters_per_epoch=10)
        tr.sched.step = lambda: None        # constant lr for the comparison
        assert isinstance(tr.model, torch.nn.parallel.DistributedDataParallel)
        tr.step_batch(_shard(d, rank), [_Sample()])
        torch.save({k: v.detach() for k, v in m.state_dict().items()}, os.path.join(out_dir, f"r{rank}.pt"))
    finally:
        dist.destroy_process_group()


def test_ddp_gloo_world2_centerpoint_matches_averaged_single_process(tmp_path):
    d = _load(TAG)
    assert int(d["coors"][:, 0].max()) + 1 == WORLD     # one frame per rank
    mp.start_processes(_worker, args=(_free_port(), str(tmp_path)), nprocs=WORLD, join=True, start_method="spawn")
    s0 = torch.load(tmp_path / "r0.pt", weights_only=True)
    s1 = torch.load(tmp_path / "r1.pt", weights_only=True)
    # single-process reference: mean of per-shard grads -> clip 0.5 -> AdamW (same groups)
    m = _build(d)
    tr = Trainer(m, lr=1e-2, ddp=False, device=torch.device("cpu"), iters_per_epoch=10)
    params = [p for p in m.parameters() if p.requires_grad]
    acc = [torch.zeros_like(p) for p in params]
    for r in range(WORLD):
        total, _ = parse_losses(m.loss(_shard(d, r), [_Sample()]))
        total.backward()
        for a, p in zip(acc, params):
            if p.grad is not None:
                a += p.grad / WORLD
        m.zero_grad(set_to_none=True)
    for a, p in zip(acc, params):
        p.grad = a
    torch.nn.utils.clip_grad_norm_(params, 0.5)
    tr.opt.step()
    ref = m.state_dict()
    # a fresh load: the stand-in head's weight is a view of the fixture's array, which the step just moved
    init = _build(_load(TAG)).state_dict()
    moved = set()
    for k in ref:
        if not torch.is_floating_point(ref[k]):
            continue
        assert torch.equal(s0[k], s1[k]), k                 # ranks agree bit-for-bit
        np.testing.assert_allclose(s0[k].double().numpy(), ref[k].double().numpy(), rtol=1e-5, atol=1e-7,
                                   err_msg=k)
        if not torch.equal(ref[k], init[k]):
            moved.add(k.split(".")[0])
    assert {"adversary", "pts_bbox_head"} <= moved, moved     # the perturber and the head both stepped
