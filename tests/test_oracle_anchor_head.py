"""oracle/anchor_head.py known-answer checks (CPU). The Anchor3DHead path has no vectors in the
reference (mmdet3d / mmcv not vendored): these pin the restatement's arithmetic on cases whose
answers follow from the upstream definitions by hand."""
import math

import numpy as np
import torch

from oracle import anchor_head as oh

CAR = dict(num_classes=1, ranges=[[0, -40.0, -1.78, 70.4, 40.0, -1.78]], sizes=[[3.9, 1.6, 1.56]],
           rotations=[0, 1.57])


def _setup(H=8, W=8):
    cfg = oh.HeadCfg(**CAR)
    anchors = oh.grid_anchors(H, W, cfg.ranges, cfg.sizes, cfg.rotations)
    return cfg, anchors


def test_gt_on_an_anchor_is_positive_with_zero_targets():
    cfg, anchors = _setup()
    a = anchors[0, 3, 5, 0, 0].clone()           # cell (h=3, w=5), rotation 0
    gb = a.view(1, 1, 7)
    gl = torch.zeros(1, 1, dtype=torch.long)
    asg, labels, lw, bt, bw, dt, npos = oh.targets(cfg, anchors, gb, gl)
    n = (3 * 8 + 5) * 2 + 0
    assert int(asg[0, n]) == 1 and int(labels[0, n]) == 0
    assert torch.allclose(bt[0, n], torch.zeros(7), atol=1e-6)
    # yaw 0 - dir_offset(-pi/2) = pi/2 -> bin floor((pi/2)/pi) = 0
    assert int(dt[0, n]) == 0
    assert float(npos) == float((asg > 0).sum())


def test_no_gt_all_negative_and_num_total_pos_clamped():
    cfg, anchors = _setup()
    gb = torch.zeros(2, 1, 7)
    gb[..., 3:6] = 1
    gl = torch.full((2, 1), -1, dtype=torch.long)
    asg, labels, lw, bt, bw, dt, npos = oh.targets(cfg, anchors, gb, gl)
    assert int((asg != 0).sum()) == 0 and float(lw.min()) == 1.0
    assert float(npos) == 2.0                     # sum_b max(0, 1)
    assert int((labels != cfg.C).sum()) == 0


def test_focal_smoothl1_and_dir_ce_values():
    x = torch.tensor([[0.3]], dtype=torch.float64)
    p = 1 / (1 + math.exp(-0.3))
    pos = float(oh.sigmoid_focal_loss(x, torch.tensor([0])))
    neg = float(oh.sigmoid_focal_loss(x, torch.tensor([1])))
    assert abs(pos - (-0.25 * (1 - p) ** 2 * math.log(p))) < 1e-12
    assert abs(neg - (-0.75 * p ** 2 * math.log(1 - p))) < 1e-12
    b = 1.0 / 9.0
    d = torch.tensor([0.05, -0.5], dtype=torch.float64)
    v = oh.smooth_l1(d, torch.zeros(2, dtype=torch.float64), b)
    assert abs(float(v[0]) - 0.5 * 0.05 ** 2 / b) < 1e-12 and abs(float(v[1]) - (0.5 - 0.5 * b)) < 1e-12


def test_low_quality_match_assigns_best_anchor():
    """A GT whose best IoU is in [min_pos_iou, pos_iou_thr) still gets its best anchor(s)
    (match_low_quality); without that rule the anchor would be ignored (-1)."""
    cfg, anchors = _setup(H=4, W=4)
    a = anchors[0, 1, 2, 0, 0].clone()
    gb = a.clone().view(1, 1, 7)
    gb[..., 4] = a[4] / 2                        # half the width: IoU = 0.5 with that anchor
    gl = torch.zeros(1, 1, dtype=torch.long)
    asg, *_ = oh.targets(cfg, anchors, gb, gl)
    ov = oh.bbox_overlaps_iou(oh.nearest_bev(gb[0]), oh.nearest_bev(anchors.reshape(-1, 7)))[0]
    assert abs(float(ov.max()) - 0.5) < 1e-6
    pos = set(np.flatnonzero(asg[0].numpy() == 1))
    assert pos == set(np.flatnonzero((ov == ov.max()).numpy())) and len(pos) >= 1


def test_fp32_and_fp64_losses_agree():
    cfg, anchors = _setup(H=16, W=16)
    g = torch.Generator().manual_seed(0)
    cls = torch.randn(2, 2, 16, 16, generator=g) - 3
    reg = torch.randn(2, 14, 16, 16, generator=g) * 0.2
    dcl = torch.randn(2, 4, 16, 16, generator=g)
    gb = anchors[0, 2:12:3, 4, 0, 0].clone().view(1, -1, 7).repeat(2, 1, 1)
    gb[..., 6] += 0.3
    gl = torch.zeros(2, gb.shape[1], dtype=torch.long)
    a = oh.losses(cfg, cls, reg, dcl, anchors, gb, gl)
    b = oh.losses(cfg, cls.double(), reg.double(), dcl.double(), anchors, gb, gl)
    for k in ("loss_cls", "loss_bbox", "loss_dir"):
        assert abs(float(a[k]) - float(b[k])) <= 1e-5 * max(1.0, abs(float(b[k])))
    assert float(a["num_total_pos"]) > 2
