"""bf16 perf mode against the fp32 parity mode over a short training trajectory:
the same 3-class model, initial weights and frames, trained 6 steps with Trainer(bf16=True) (16-bit
MFMA sparse layers 1-11 — fp16 forward operands, bf16 backward — bf16 SECOND/FPN/head GEMMs) and
Trainer(bf16=False) (fp32 HIP kernels end to end). Per step the detection losses and the total agree within the pinned bounds below, and the
adversary's parameter updates (what the perturber learns) point the same way. Bench numbers are
bf16 perf-mode numbers; this test bounds how far that mode drifts from the parity mode."""
import pytest
import torch

from robustpointclouds_amd.anchor_head import pack_gt
from robustpointclouds_amd.synthetic import kitti_batch
from robustpointclouds_amd.trainer import Trainer, make_kitti_model

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")
STEPS = 6
# r04: with the sparse encoder's forward GEMM operands in fp16 (SparseEncoder FWD_FMT; r02/r03 bf16: loss rel
# 1.05e-2, adversary cosine 0.9915) measured 6.6e-3 and 0.99550
LOSS_REL = 1e-2      # per-step |perf - fp32| / |fp32| of loss_cls, loss_bbox, loss_dir and the total
ADV_COS = 0.995      # cosine of the adversary's parameter change (perf vs fp32) after STEPS steps


def _run(bf16, batches):
    torch.manual_seed(5)
    model = make_kitti_model(num_classes=3, device=DEV, epoch=3)
    p0 = {k: v.detach().clone() for k, v in model.adversary.named_parameters()}
    tr = Trainer(model, bf16=bf16, device=DEV)
    logs = []
    for pts, gt in batches:
        lg = tr.train_step(pts, gt)
        logs.append({k: float(v) for k, v in lg.items()})
    dp = torch.cat([(v.detach() - p0[k]).flatten() for k, v in model.adversary.named_parameters()])
    return logs, dp


def test_bf16_tracks_fp32_trajectory():
    batches = []
    for s in range(STEPS):
        pts, boxes, labels = kitti_batch(4, seed0=900 + 4 * s, num_classes=3)
        gb, gl = pack_gt(list(zip(boxes, labels)), DEV)
        batches.append(([torch.from_numpy(p).to(DEV) for p in pts], dict(gt_boxes=gb, gt_labels=gl)))
    l16, d16 = _run(True, batches)
    l32, d32 = _run(False, batches)
    worst = 0.0
    for s, (a, b) in enumerate(zip(l16, l32)):
        for k in ("loss_cls", "loss_bbox", "loss_dir", "loss"):
            rel = abs(a[k] - b[k]) / max(abs(b[k]), 1e-6)
            worst = max(worst, rel)
            assert rel <= LOSS_REL, (s, k, a[k], b[k], rel)
    cos = float(d16 @ d32 / (d16.norm() * d32.norm()).clamp_min(1e-30))
    print(f"bf16 vs fp32 over {STEPS} steps: worst loss rel {worst:.3e}, adversary update cosine {cos:.5f}")
    assert cos >= ADV_COS, cos
