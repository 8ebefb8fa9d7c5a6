"""PARITY ORACLE — TEST INFRASTRUCTURE ONLY (tests/, bench cpu_baseline).

CPU restatement of the Anchor3DHead training targets and losses (SURVEY.md §8(a) row a8,
§8(f1)), in explicit torch ops (float64 by default; float32 keeps the reference's op order):

* anchors      upstream mmdet3d `Anchor3DRangeGenerator.anchors_single_range` (torch.linspace
               centres, [D, H, W, S, R, 7], sizes/rotations as configured)
* nearest_bev  `BaseInstance3DBoxes.nearest_bev`; IoU = mmdet `bbox_overlaps(mode='iou', eps=1e-6)`
               (BboxOverlapsNearest3D)
* assign       mmdet `MaxIoUAssigner.assign_wrt_overlaps` (match_low_quality, gt_max_assign_all:
               later GTs overwrite), one assigner per anchor size for list-valued train_cfg.assigner
               (`AnchorTrainMixin.anchor_target_single`, assign_per_class optional)
* targets      `anchor_target_single_assigner`: DeltaXYZWLHRBBoxCoder.encode, get_direction_target,
               label_weights (pos_weight), num_total_pos = sum_b max(pos_b, 1)
* losses       mmcv sigmoid_focal_loss (mmdet FocalLoss, sigmoid, gamma 2, alpha 0.25), mmdet
               SmoothL1Loss (beta 1/9, x2) with add_sin_difference, CrossEntropyLoss (x0.2) on the
               positives, each / (num_total_pos + eps) — `Anchor3DHead.loss_by_feat_single`

as configured at configs/adversarial/adversarial-second_hv_secfpn_8xb6-80e_kitti-3d-3class.py:38-69,
:86-112 and …-kitti-3d-car.py:18-39 (head called at models/detectors/adversarial_voxelnet.py:168).
mmdet3d / mmdet / mmcv are not vendored in /root/reference and no reference test holds vectors for
this row: parity is UNPINNED w.r.t. upstream (the restatement follows the published v1.x
semantics). Gradients are taken by torch autograd of these expressions.
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn.functional as Fn

FLT_MIN = 1.1754943508222875e-38
EPS = float(torch.finfo(torch.float32).eps)


def limit_period(val, offset=0.5, period=math.pi):
    return val - torch.floor(val / period + offset) * period


def anchors_single_range(feature_size, anchor_range, sizes, rotations, dtype=torch.float32):
    """[D, H, W, S, R, 7] anchors of one range (Anchor3DRangeGenerator.anchors_single_range)."""
    if len(feature_size) == 2:
        feature_size = [1, feature_size[0], feature_size[1]]
    r = torch.tensor(anchor_range, dtype=torch.float32)
    zc = torch.linspace(r[2], r[5], feature_size[0])
    yc = torch.linspace(r[1], r[4], feature_size[1])
    xc = torch.linspace(r[0], r[3], feature_size[2])
    sizes = torch.tensor(sizes, dtype=torch.float32).reshape(-1, 3)
    rot = torch.tensor(rotations, dtype=torch.float32)
    rets = list(torch.meshgrid(xc, yc, zc, rot, indexing="ij"))
    tile = [1] * 5
    tile[-2] = int(sizes.shape[0])
    for i in range(len(rets)):
        rets[i] = rets[i].unsqueeze(-2).repeat(tile).unsqueeze(-1)
    sizes = sizes.reshape([1, 1, 1, -1, 1, 3])
    ts = list(rets[0].shape)
    ts[3] = 1
    rets.insert(3, sizes.repeat(ts))
    return torch.cat(rets, dim=-1).permute([2, 1, 0, 3, 4, 5]).to(dtype)


def grid_anchors(H, W, ranges, sizes, rotations, dtype=torch.float32):
    """[1, H, W, S, R, 7]: one range per size (size_per_range), concatenated on the size axis."""
    if len(sizes) == 1 and len(ranges) > 1:
        sizes = sizes * len(ranges)
    return torch.cat([anchors_single_range([H, W], rg, [sz], rotations, dtype) for rg, sz in zip(ranges, sizes)],
                     dim=-3)


def nearest_bev(boxes):
    bev = boxes[..., [0, 1, 3, 4, 6]]
    nr = torch.abs(limit_period(bev[..., -1], 0.5, np.pi))
    cond = (nr > np.pi / 4)[..., None]
    xywh = torch.where(cond, bev[..., [0, 1, 3, 2]], bev[..., :4])
    c, d = xywh[..., :2], xywh[..., 2:]
    return torch.cat([c - d / 2, c + d / 2], dim=-1)


def bbox_overlaps_iou(b1, b2, eps=1e-6):
    a1 = (b1[..., 2] - b1[..., 0]) * (b1[..., 3] - b1[..., 1])
    a2 = (b2[..., 2] - b2[..., 0]) * (b2[..., 3] - b2[..., 1])
    lt = torch.max(b1[..., :, None, :2], b2[..., None, :, :2])
    rb = torch.min(b1[..., :, None, 2:], b2[..., None, :, 2:])
    wh = (rb - lt).clamp(min=0)
    ov = wh[..., 0] * wh[..., 1]
    union = torch.clamp(a1[..., None] + a2[..., None, :] - ov, min=eps)
    return ov / union


def assign_max_iou(anchors_bev, gt_bev, gt_valid, pos_thr, neg_thr, min_pos):
    """[B, A] assignment: 0 neg, -1 ignore, j+1 positive for gt j."""
    ov = bbox_overlaps_iou(gt_bev, anchors_bev.expand(gt_bev.shape[0], -1, -1))   # [B, M, A]
    ov = torch.where(gt_valid[..., None], ov, torch.full_like(ov, -1.0))
    max_ov, argmax = ov.max(dim=1)
    gt_max, _ = ov.max(dim=2)
    assigned = torch.full_like(argmax, -1)
    assigned = torch.where((max_ov >= 0) & (max_ov < neg_thr), torch.zeros_like(assigned), assigned)
    assigned = torch.where(max_ov >= pos_thr, argmax + 1, assigned)
    M = ov.shape[1]
    lowq = (gt_max[..., None] >= min_pos) & (ov == gt_max[..., None]) & gt_valid[..., None]
    gi = torch.arange(M).view(1, M, 1).expand_as(ov)
    last = torch.where(lowq, gi, torch.full_like(gi, -1)).max(dim=1).values
    assigned = torch.where(last >= 0, last + 1, assigned)
    no_gt = ~gt_valid.any(dim=1, keepdim=True)
    return torch.where(no_gt, torch.zeros_like(assigned), assigned)


def encode(src, dst):
    xa, ya, za, wa, la, ha, ra = torch.split(src, 1, dim=-1)
    xg, yg, zg, wg, lg, hg, rg = torch.split(dst, 1, dim=-1)
    za = za + ha / 2
    zg = zg + hg / 2
    diag = torch.sqrt(la ** 2 + wa ** 2)
    return torch.cat([(xg - xa) / diag, (yg - ya) / diag, (zg - za) / ha, torch.log(wg / wa),
                      torch.log(lg / la), torch.log(hg / ha), rg - ra], dim=-1)


def sigmoid_focal_loss(pred, target, gamma=2.0, alpha=0.25):
    C = pred.shape[-1]
    p = torch.sigmoid(pred)
    t = Fn.one_hot(target.clamp(max=C), C + 1)[..., :C].to(pred.dtype)
    pos = -alpha * torch.pow(1.0 - p, gamma) * torch.log(torch.clamp(p, min=FLT_MIN))
    neg = -(1.0 - alpha) * torch.pow(p, gamma) * torch.log(torch.clamp(1.0 - p, min=FLT_MIN))
    return t * pos + (1.0 - t) * neg


def smooth_l1(pred, target, beta):
    diff = torch.abs(pred - target)
    return torch.where(diff < beta, 0.5 * diff * diff / beta, diff - 0.5 * beta)


def add_sin_difference(b1, b2):
    rp = torch.sin(b1[..., 6:7]) * torch.cos(b2[..., 6:7])
    rt = torch.cos(b1[..., 6:7]) * torch.sin(b2[..., 6:7])
    return (torch.cat([b1[..., :6], rp, b1[..., 7:]], dim=-1), torch.cat([b2[..., :6], rt, b2[..., 7:]], dim=-1))


class HeadCfg:
    """The Anchor3DHead settings the restatement needs (defaults: SECOND KITTI configs)."""

    def __init__(self, num_classes, ranges, sizes, rotations=(0, 1.57), assigners=None, assign_per_class=False,
                 pos_weight=-1.0, dir_offset=-np.pi / 2, dir_limit_offset=0.0, diff_rad_by_sin=True,
                 use_dir=True, gamma=2.0, alpha=0.25, beta=1.0 / 9.0, lw_cls=1.0, lw_bbox=2.0, lw_dir=0.2):
        self.C = num_classes
        self.ranges, self.sizes, self.rotations = [list(r) for r in ranges], [list(s) for s in sizes], list(rotations)
        assigners = assigners or [dict(pos_iou_thr=0.6, neg_iou_thr=0.45, min_pos_iou=0.45)]
        self.assigners = assigners if isinstance(assigners, (list, tuple)) else [assigners]
        self.assigner_is_list = isinstance(assigners, (list, tuple)) and len(self.assigners) > 1
        self.assign_per_class = assign_per_class
        self.pos_weight, self.dir_offset, self.dir_limit_offset = pos_weight, dir_offset, dir_limit_offset
        self.diff_rad_by_sin, self.use_dir = diff_rad_by_sin, use_dir
        self.gamma, self.alpha, self.beta = gamma, alpha, beta
        self.lw_cls, self.lw_bbox, self.lw_dir = lw_cls, lw_bbox, lw_dir

    @property
    def S(self):
        return max(len(self.ranges), len(self.sizes))

    @property
    def R(self):
        return len(self.rotations)


def cfg_of(head) -> HeadCfg:
    """HeadCfg from an Anchor3DHead-like module (duck-typed: prior_generator, assigners, loss cfgs)."""
    g = head.prior_generator
    tc = getattr(head, "train_cfg", {}) or {}
    return HeadCfg(head.num_classes, g.ranges, g.sizes, g.rotations,
                   head.assigners if head.assigner_is_list else head.assigners[0],
                   assign_per_class=head.assign_per_class, pos_weight=float(tc.get("pos_weight", -1)),
                   dir_offset=head.dir_offset, dir_limit_offset=head.dir_limit_offset,
                   diff_rad_by_sin=head.diff_rad_by_sin, use_dir=head.use_direction_classifier,
                   gamma=head.loss_cls_cfg.get("gamma", 2.0), alpha=head.loss_cls_cfg.get("alpha", 0.25),
                   beta=head.loss_bbox_cfg.get("beta", 1.0 / 9.0), lw_cls=head.loss_cls_cfg.get("loss_weight", 1.0),
                   lw_bbox=head.loss_bbox_cfg.get("loss_weight", 2.0), lw_dir=head.loss_dir_cfg.get("loss_weight", 0.2))


def targets(cfg: HeadCfg, anchors, gt_boxes, gt_labels):
    """anchor_target_3d over a batch. anchors [1, H, W, S, R, 7]; gt_boxes [B, M, 7], gt_labels [B, M]
    (-1 padding). Returns (assigned [B, N], labels, label_w, bbox_t [B, N, 7], bbox_w, dir_t, npos),
    N = H*W*S*R in the channel order of the head outputs (cell-major, then size, then rotation)."""
    valid = gt_labels >= 0
    gt_bev = nearest_bev(gt_boxes)
    S, R = anchors.size(-3), anchors.size(-2)
    A_flat = anchors.reshape(-1, 7)
    if cfg.assigner_is_list:
        assert S == len(cfg.assigners)
        parts = []
        for i, a in enumerate(cfg.assigners):
            an = anchors[..., i, :, :].reshape(-1, 7)
            gv = valid & (gt_labels == i) if cfg.assign_per_class else valid
            parts.append(assign_max_iou(nearest_bev(an), gt_bev, gv, a["pos_iou_thr"], a["neg_iou_thr"],
                                        a["min_pos_iou"]))
        asg = torch.stack([p.view(p.shape[0], -1, R) for p in parts], dim=2).reshape(gt_boxes.shape[0], -1)
    else:
        a = cfg.assigners[0]
        asg = assign_max_iou(nearest_bev(A_flat), gt_bev, valid, a["pos_iou_thr"], a["neg_iou_thr"], a["min_pos_iou"])
    B, N = asg.shape
    pos, neg = asg > 0, asg == 0
    gidx = (asg - 1).clamp(min=0)
    matched = torch.gather(gt_boxes, 1, gidx[..., None].expand(B, N, 7))
    mlabel = torch.gather(gt_labels, 1, gidx)
    anc = A_flat.unsqueeze(0).expand(B, N, 7)
    bbox_t = encode(anc, matched)
    bbox_t = torch.where(pos[..., None], bbox_t, torch.zeros_like(bbox_t))
    rot_gt = bbox_t[..., 6] + anc[..., 6]
    off = limit_period(rot_gt - cfg.dir_offset, cfg.dir_limit_offset, 2 * np.pi)
    dir_t = torch.floor(off / (2 * np.pi / 2)).long().clamp(0, 1)
    dir_t = torch.where(pos, dir_t, torch.zeros_like(dir_t))
    labels = torch.where(pos, mlabel, torch.full_like(mlabel, cfg.C))
    pw = cfg.pos_weight
    label_w = torch.where(pos, torch.full_like(asg, 1, dtype=anchors.dtype) * (1.0 if pw <= 0 else pw),
                          neg.to(anchors.dtype))
    npos = pos.sum(dim=1).clamp(min=1).sum().to(anchors.dtype)
    return asg, labels, label_w, bbox_t, pos.to(anchors.dtype), dir_t, npos


def losses(cfg: HeadCfg, cls, reg, dcl, anchors, gt_boxes, gt_labels):
    """Anchor3DHead.loss_by_feat for one level: cls [B, A*C, H, W], reg [B, A*7, H, W],
    dcl [B, A*2, H, W] -> dict(loss_cls, loss_bbox, loss_dir, num_total_pos, assigned).
    Targets are computed in float32 from float32 anchors / GT boxes, as the reference does; the
    losses in the dtype of the predictions (float64 for an accurate reference)."""
    asg, labels, label_w, bbox_t, bbox_w, dir_t, npos = targets(cfg, anchors.float(), gt_boxes.float(), gt_labels)
    dt = cls.dtype
    label_w, bbox_t, bbox_w, npos = label_w.to(dt), bbox_t.to(dt), bbox_w.to(dt), npos.to(dt)
    C = cfg.C
    cs = cls.permute(0, 2, 3, 1).reshape(-1, C)
    lc = sigmoid_focal_loss(cs, labels.reshape(-1), cfg.gamma, cfg.alpha)
    loss_cls = (lc * label_w.reshape(-1, 1)).sum() / (npos + EPS) * cfg.lw_cls
    bp = reg.permute(0, 2, 3, 1).reshape(-1, 7)
    bt = bbox_t.reshape(-1, 7)
    bw = bbox_w.reshape(-1, 1).expand_as(bt)
    if cfg.diff_rad_by_sin:
        bp, bt = add_sin_difference(bp, bt)
    loss_bbox = (smooth_l1(bp, bt, cfg.beta) * bw).sum() / (npos + EPS) * cfg.lw_bbox
    out = dict(loss_cls=loss_cls, loss_bbox=loss_bbox, num_total_pos=npos, assigned=asg)
    if cfg.use_dir:
        dp = dcl.permute(0, 2, 3, 1).reshape(-1, 2)
        ce = Fn.cross_entropy(dp, dir_t.reshape(-1), reduction="none")
        out["loss_dir"] = (ce * bbox_w.reshape(-1)).sum() / (npos + EPS) * cfg.lw_dir
    return out


def head_losses_from_z(cfg: HeadCfg, z, bias, anchors, gt_boxes, gt_labels):
    """z [B, N, H, W] raw 1x1-conv outputs (cls | reg | dir channel groups), bias [N]."""
    A = cfg.S * cfg.R
    y = z + bias.view(1, -1, 1, 1)
    cls, reg, dcl = torch.split(y, [A * cfg.C, A * 7, A * 2 if cfg.use_dir else 0], dim=1)
    return losses(cfg, cls, reg, dcl, anchors, gt_boxes, gt_labels)
