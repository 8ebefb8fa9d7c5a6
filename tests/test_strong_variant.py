"""§8(f4) StrongAdversarialVoxelNet (BASELINE config 5) against golden vectors from the reference's
own class (tests/golden/make_golden.py:gen_strong; models/detectors/strong_adversarial_voxelnet.py).

Fixtures: `list` / `tensor` — constant V (cross-step momentum), list- / tensor-valued head losses;
`weak` / `tiny` — V alternating (momentum reset on every shape change) with small l2, so the
attack-history boost engages after 50 steps (x1.5 and x2). Every fixture runs 53-56 loss() calls with
the torch host RNG seeded for the anti-adaptation draws; per-step losses, l2 and scaling are
compared, and the final step's parameter gradients.

* CPU: oracle/strong.py (OraclePerturber adversary) — pins the restatement.
* GPU: the plugin StrongAdversarialVoxelNet (HIP VoxelPerturber + HIP HardSimpleVFE + the
  csrc/strong.hip combine kernel) — values within 1e-4 relative (north_star fp32 tolerance).
"""
import os

import numpy as np
import pytest
import torch
from torch import nn

from oracle.perturber import OraclePerturber
from oracle.strong import OracleStrong
from tests.conftest import GOLDEN
from tests.test_adversarial_voxelnet import StandInHead, StandInMiddle, StandInVFE

TAGS = ["list", "tensor", "weak", "tiny"]
KEYS = ("loss_cls", "loss_bbox", "loss_dir", "loss_adversarial", "loss_l2_regularization")


def _load(tag):
    return dict(np.load(os.path.join(GOLDEN, f"strong_{tag}.npz")))


def _inputs(d, step, dev):
    k = step % int(d["nsets"])
    return {"voxels": {"voxels": torch.from_numpy(d[f"vox{k}"]).to(dev),
                       "num_points": torch.from_numpy(d[f"num_points{k}"]).to(dev),
                       "coors": torch.from_numpy(d[f"coors{k}"]).to(dev)}, "batch_size": 2}


def _val(v):
    return float((v[0] if isinstance(v, list) else v).detach().cpu())


def _total(losses):
    t = 0
    for k, v in losses.items():
        if "loss" in k:
            t = t + (sum(x.mean() for x in v) if isinstance(v, list) else v.mean())
    return t


@pytest.mark.parametrize("tag", TAGS)
def test_oracle_strong_matches_reference(tag):
    d = _load(tag)
    hidden = [int(h) for h in d["hidden"]]
    op = OraclePerturber(d, 4, hidden, dtype=torch.float32, sensor_error_bound=float(d["bound"]))

    def adversary(x):
        out, ld = op.forward(x)
        return out.to(x.dtype), ld

    o = OracleStrong(adversary)
    o.epoch = int(d["epoch"])
    vfe, mid, head = StandInVFE(), StandInMiddle(), StandInHead(d["head_w"], bool(d["listy"]))
    torch.manual_seed(int(d["seed"]))
    for step in range(int(d["steps"])):
        vd = _inputs(d, step, "cpu")["voxels"]
        feats = vfe(vd["voxels"], vd["num_points"], vd["coors"])
        losses, l2 = o.loss(feats, vd["coors"], 2, mid, nn.Identity(), head, None)
        for k in KEYS:
            np.testing.assert_allclose(_val(losses[k]), d["S_" + k][step], rtol=2e-5, atol=1e-7, err_msg=f"{k}@{step}")
        np.testing.assert_allclose(float(l2), d["S_l2"][step], rtol=2e-5)
        np.testing.assert_allclose(o.scaling, d["S_scaling"][step], rtol=1e-12)
    _total(losses).backward()
    g = op.grads()
    for l in range(6):
        np.testing.assert_allclose(g[f"dW{l}"].numpy(), d[f"dW{l}"], rtol=0, atol=1e-4 * max(1e-3, np.abs(d[f"dW{l}"]).max()))
    np.testing.assert_allclose(head.w.grad.numpy(), d["dhead_w"], rtol=1e-4, atol=1e-7)


@pytest.mark.gpu
@pytest.mark.parametrize("tag", TAGS)
def test_hip_strong_matches_reference(tag):
    import robustpointclouds_amd.plugin.models  # noqa: F401
    from robustpointclouds_amd.plugin.models.adversarial.voxel_perturber import VoxelPerturber
    from robustpointclouds_amd.plugin.models.detectors.strong_adversarial_voxelnet import StrongAdversarialVoxelNet
    from robustpointclouds_amd.voxelnet import HardSimpleVFE
    from tests.test_adversarial_voxelnet import _set_weights

    d = _load(tag)
    dev = torch.device("cuda")
    hidden = [int(h) for h in d["hidden"]]
    m = StrongAdversarialVoxelNet(
        voxel_encoder=HardSimpleVFE(), middle_encoder=StandInMiddle(), backbone=nn.Identity(), neck=None,
        bbox_head=StandInHead(d["head_w"], bool(d["listy"])),
        adversary_cfg=dict(type="VoxelPerturber", sensor_error_bound=float(d["bound"]), hidden_channels=hidden)).to(dev)
    assert isinstance(m.adversary, VoxelPerturber)
    _set_weights(m.adversary, d)
    m.train()
    m._epoch = int(d["epoch"])
    torch.manual_seed(int(d["seed"]))
    for step in range(int(d["steps"])):
        inputs = _inputs(d, step, dev)
        losses = m.loss(inputs, None)
        for k in KEYS:
            np.testing.assert_allclose(_val(losses[k]), d["S_" + k][step], rtol=1e-4, atol=1e-6, err_msg=f"{k}@{step}")
        np.testing.assert_allclose(float(inputs["adversarial_l2_norm"]), d["S_l2"][step], rtol=1e-4)
        np.testing.assert_allclose(m._current_scaling, d["S_scaling"][step], rtol=1e-6)
    _total(losses).backward()
    lin = [mod for mod in m.adversary.model if isinstance(mod, nn.Linear)]
    for l, mod in enumerate(lin):
        ref = d[f"dW{l}"]
        np.testing.assert_allclose(mod.weight.grad.cpu().numpy(), ref, rtol=0, atol=1e-3 * max(1e-3, np.abs(ref).max()))
    np.testing.assert_allclose(m.bbox_head.w.grad.cpu().numpy(), d["dhead_w"], rtol=1e-3, atol=1e-6)


@pytest.mark.gpu
@pytest.mark.parametrize("bf16", [True, False])
def test_strong_full_model_config5(bf16):
    """BASELINE config 5 on the full model: StrongAdversarialVoxelNet (sensor_error_bound 0.4) with the real
    SECOND stack (HardSimpleVFE, SparseEncoder, SECOND / SECONDFPN, Anchor3DHead) at the config's batch, 6
    synthetic KITTI frames, 3 classes, three Trainer steps (bf16 perf mode and fp32 parity mode). The
    combination itself is pinned by the fixture tests above; here: the reference's loss keys
    (strong_adversarial_voxelnet.py:254-303), finite values, the adversarial term of list-valued head losses, the dynamic scaling
    within [1, max_scaling], the cross-step momentum engaged, and every stage's parameters moved."""
    from robustpointclouds_amd.anchor_head import pack_gt
    from robustpointclouds_amd.plugin.models.detectors.strong_adversarial_voxelnet import StrongAdversarialVoxelNet
    from robustpointclouds_amd.synthetic import kitti_batch
    from robustpointclouds_amd.trainer import Trainer, make_kitti_model

    dev = torch.device("cuda")
    torch.manual_seed(5)
    model = make_kitti_model(num_classes=3, device=dev, epoch=3, variant="strong")
    assert isinstance(model, StrongAdversarialVoxelNet)
    assert abs(model.adversary.sensor_error_bound - 0.4) < 1e-12
    tr = Trainer(model, bf16=bf16, device=dev)
    before = {k: v.detach().clone() for k, v in model.named_parameters()}
    pts, boxes, labels = kitti_batch(6, seed0=700, num_classes=3)
    gpts = [torch.from_numpy(p).to(dev) for p in pts]
    gb, gl = pack_gt(list(zip(boxes, labels)), dev)
    for step in range(3):
        lg = tr.train_step(gpts, dict(gt_boxes=gb, gt_labels=gl))
        torch.cuda.synchronize()
        vals = {k: float(v[0] if isinstance(v, (list, tuple)) else v) for k, v in lg.items()}
        assert set(KEYS) <= set(vals), sorted(vals)
        assert all(np.isfinite(v) for v in vals.values()), vals
        # the Anchor3DHead's losses are per-level lists, which the reference's tensor-only detection sum skips
        # (strong_adversarial_voxelnet.py:264-267): the adversarial term is then 0 (fixture `list` pins this)
        assert vals["loss_adversarial"] == 0.0, vals
        assert vals["loss_l2_regularization"] > 0, vals
        s = model._current_scaling
        assert 1.0 <= s <= model.max_scaling, s
    assert model._attack_count == 3 and model._last_adversarial_loss is not None
    moved = {k.split(".")[0] for k, v in model.named_parameters() if not torch.equal(v.detach(), before[k])}
    assert {"adversary", "middle_encoder", "backbone", "neck", "bbox_head"} <= moved, moved
