"""§8(f3): AdversarialCenterPoint training steps end to end on the HIP stack (voxelize F=5 ->
fused perturber + VFE -> basicblock SparseEncoder -> SECOND/FPN -> DCN CenterHead -> CenterHead
losses -> adversarial combination -> ClipAdamW), synthetic 3-sweep nuScenes-like frames.

Checks the reference's loss keys (task{t}.loss_heatmap / loss_bbox, loss_adversarial,
loss_l2_regularization, perturbation_l2_norm — adversarial_centerpoint.py:224-257), the adversarial
combination (-min(w * epoch / 10, w) * sum of the [0, 100]-clamped detection losses, the l2 term),
the epoch < 3 gate (:66), finite values and that the parameters move."""
import pytest
import torch

from robustpointclouds_amd.center_head import pack_gt
from robustpointclouds_amd.synthetic import nus_frame, nus_gt_boxes
from robustpointclouds_amd.trainer import Trainer, make_nus_model

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


def _batch(B, seed, sweeps=3):
    pts = [torch.from_numpy(nus_frame(seed + i, sweeps=sweeps)).to(DEV) for i in range(B)]
    gts = [nus_gt_boxes(seed + i) for i in range(B)]
    gb, gl = pack_gt([torch.from_numpy(b) for b, _ in gts], [torch.from_numpy(l) for _, l in gts], DEV)
    return pts, dict(gt_boxes=gb, gt_labels=gl)


@pytest.mark.parametrize("bf16", [True, False])
def test_adversarial_centerpoint_steps(bf16):
    """bf16 perf mode and the fp32 parity mode (fp32 perturber, 128-wide fp32 sparse convs, fp32 dense
    engine, fp32 DCN and head images)."""
    torch.manual_seed(0)
    model = make_nus_model(device=DEV, epoch=3)
    tr = Trainer(model, bf16=bf16, device=DEV)
    before = {k: v.detach().clone() for k, v in model.named_parameters()}
    pts, gt = _batch(2, 0)
    logs = [tr.train_step(pts, gt) for _ in range(3)]
    torch.cuda.synchronize()
    want = {f"task{t}.{k}" for t in range(6) for k in ("loss_heatmap", "loss_bbox")} | \
        {"loss_adversarial", "loss_l2_regularization", "perturbation_l2_norm"}
    for lg in logs:
        assert want <= set(lg), sorted(set(lg))
        vals = {k: float(v) for k, v in lg.items()}
        assert all(torch.isfinite(torch.tensor(v)) for v in vals.values()), vals
        det = sum(min(max(vals[k], 0.0), 100.0) for k in want if k.startswith("task"))
        w = min(0.05 * 3 / 10, 0.05)
        assert abs(vals["loss_adversarial"] - (-w * det)) <= 1e-4 * max(1.0, det)
        assert abs(vals["loss_l2_regularization"] - 0.005 * vals["perturbation_l2_norm"]) <= 1e-6
        assert vals["perturbation_l2_norm"] > 0
    moved = [k for k, v in model.named_parameters() if not torch.equal(v.detach(), before[k])]
    assert any(k.startswith("adversary") for k in moved)
    assert any(k.startswith("pts_bbox_head.task_heads.5") for k in moved)
    assert any(k.startswith("pts_middle_encoder.encoder_layers.encoder_layer4") for k in moved)


def test_gate_closed_before_epoch_3():
    torch.manual_seed(0)
    model = make_nus_model(device=DEV, epoch=2)
    tr = Trainer(model, bf16=True, device=DEV)
    pts, gt = _batch(1, 7)
    lg = tr.train_step(pts, gt)
    assert float(lg["loss_adversarial"]) == 0.0 and float(lg["loss_l2_regularization"]) == 0.0
    assert "perturbation_l2_norm" not in lg


def test_adversarial_centerpoint_config_size():
    """BASELINE config 4 at its own size: batch 4 per GPU, 10-sweep nuScenes-like frames (~240k
    points each, 90000-voxel cap at 0.1 m), two training steps in bf16 perf mode: the reference's
    loss keys, finite values, the adversarial combination and the l2 term."""
    torch.manual_seed(1)
    model = make_nus_model(device=DEV, epoch=3)
    tr = Trainer(model, bf16=True, device=DEV)
    pts, gt = _batch(4, 40, sweeps=10)
    assert all(p.shape[0] > 150000 for p in pts), [p.shape[0] for p in pts]
    want = {f"task{t}.{k}" for t in range(6) for k in ("loss_heatmap", "loss_bbox")} | \
        {"loss_adversarial", "loss_l2_regularization", "perturbation_l2_norm"}
    for _ in range(2):
        lg = tr.train_step(pts, gt)
        vals = {k: float(v) for k, v in lg.items()}
        assert want <= set(lg), sorted(set(lg))
        assert all(torch.isfinite(torch.tensor(v)) for v in vals.values()), vals
        det = sum(min(max(vals[k], 0.0), 100.0) for k in want if k.startswith("task"))
        assert abs(vals["loss_adversarial"] - (-0.015 * det)) <= 1e-4 * max(1.0, det)
        assert abs(vals["loss_l2_regularization"] - 0.005 * vals["perturbation_l2_norm"]) <= 1e-6
