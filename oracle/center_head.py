"""PARITY ORACLE — TEST INFRASTRUCTURE ONLY (tests/, bench cpu_baseline).

CPU restatement of the CenterHead training targets and losses of AdversarialCenterPoint (SURVEY.md
§8(f3), BASELINE config 4; head called at models/detectors/adversarial_centerpoint.py:210,224 with
the upstream base configs/adversarial/adversarial-centerpoint_voxel-nuscenes.py:11-13):

* targets   upstream mmdet3d `CenterHead.get_targets_single`: boxes re-ordered per task (class order
            within the task, then GT order), gravity-centre z, `gaussian_radius(min_overlap=0.1)`,
            radius = max(min_radius, int(r)), `draw_heatmap_gaussian` (float64 numpy gaussian, sigma =
            diameter / 6, max-combined, cast to float32), ind = y * W + x, mask, and the 10-value
            anno box [dx, dy, z, log(w, l, h), sin(rot), cos(rot), vx, vy]
* losses    `CenterHead.loss_by_feat`: clamp_sigmoid (1e-4), mmdet GaussianFocalLoss (alpha 2,
            gamma 4, eps 1e-12) / (max(num_pos, 1) + FLT_EPS); mmdet L1Loss on the gathered boxes with
            mask * isnotnan * code_weights, / (num + 1e-4 + FLT_EPS), x loss_weight 0.25

mmdet3d / mmdet are not vendored in /root/reference (the mmdetection3d submodule is empty) and no
reference test holds vectors for this head: parity is UNPINNED w.r.t. upstream (this follows the
published mmdet3d v1.x / mmdet v3.x semantics, float32 op order kept where it decides results).
Gradients are taken by torch autograd of these expressions.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np
import torch

FLT_EPS = float(torch.finfo(torch.float32).eps)

NUS_TASKS = (("car",), ("truck", "construction_vehicle"), ("bus", "trailer"), ("barrier",),
             ("motorcycle", "bicycle"), ("pedestrian", "traffic_cone"))


@dataclass
class CenterCfg:
    """train_cfg.pts + head settings of centerpoint_voxel01_second_secfpn_head-dcn (nuScenes)."""
    tasks: tuple = NUS_TASKS
    grid_size: tuple = (1024, 1024, 40)
    voxel_size: tuple = (0.1, 0.1, 0.2)
    point_cloud_range: tuple = (-51.2, -51.2, -5.0, 51.2, 51.2, 3.0)
    out_size_factor: int = 8
    dense_reg: int = 1
    gaussian_overlap: float = 0.1
    max_objs: int = 500
    min_radius: int = 2
    code_weights: tuple = (1.0, 1.0, 1.0, 1.0, 1.0, 1.0, 1.0, 1.0, 0.2, 0.2)
    norm_bbox: bool = True
    loss_cls_weight: float = 1.0
    loss_bbox_weight: float = 0.25

    @property
    def ncls(self):
        return [len(t) for t in self.tasks]

    @property
    def feature_map_size(self):            # (x, y) as grid_size[:2] // out_size_factor
        return (self.grid_size[0] // self.out_size_factor, self.grid_size[1] // self.out_size_factor)


def gaussian_radius(det_size, min_overlap=0.5):
    """mmdet3d `gaussian_radius` on float32 0-d tensors (python-scalar constants as torch applies them)."""
    height, width = det_size
    a1 = 1
    b1 = height + width
    c1 = width * height * (1 - min_overlap) / (1 + min_overlap)
    sq1 = torch.sqrt(b1 ** 2 - 4 * a1 * c1)
    r1 = (b1 + sq1) / 2
    a2 = 4
    b2 = 2 * (height + width)
    c2 = (1 - min_overlap) * width * height
    sq2 = torch.sqrt(b2 ** 2 - 4 * a2 * c2)
    r2 = (b2 + sq2) / 2
    a3 = 4 * min_overlap
    b3 = -2 * min_overlap * (height + width)
    c3 = (min_overlap - 1) * width * height
    sq3 = torch.sqrt(b3 ** 2 - 4 * a3 * c3)
    r3 = (b3 + sq3) / 2
    return min(r1, r2, r3)


def gaussian_2d(shape, sigma=1.0):
    m, n = [(ss - 1.0) / 2.0 for ss in shape]
    y, x = np.ogrid[-m:m + 1, -n:n + 1]
    h = np.exp(-(x * x + y * y) / (2 * sigma * sigma))
    h[h < np.finfo(h.dtype).eps * h.max()] = 0
    return h


def draw_heatmap_gaussian(heatmap, center, radius, k=1):
    diameter = 2 * radius + 1
    gaussian = gaussian_2d((diameter, diameter), sigma=diameter / 6)
    x, y = int(center[0]), int(center[1])
    height, width = heatmap.shape[0:2]
    left, right = min(x, radius), min(width - x, radius + 1)
    top, bottom = min(y, radius), min(height - y, radius + 1)
    masked_heatmap = heatmap[y - top:y + bottom, x - left:x + right]
    masked_gaussian = torch.from_numpy(gaussian[radius - top:radius + bottom,
                                                radius - left:radius + right]).to(torch.float32)
    if min(masked_gaussian.shape) > 0 and min(masked_heatmap.shape) > 0:
        torch.max(masked_heatmap, masked_gaussian * k, out=masked_heatmap)
    return heatmap


def gravity_center_boxes(boxes):
    """[N, 9] LiDAR boxes (bottom centre) -> gravity centre + the rest (`torch.cat((gravity_center,
    tensor[:, 3:]))`)."""
    b = boxes.clone()
    b[:, 2] = boxes[:, 2] + boxes[:, 5] * 0.5
    return b


def targets_single(cfg: CenterCfg, gt_boxes, gt_labels):
    """get_targets_single for one sample: per task (heatmap [ncls, H, W], anno_box [max_objs, 10],
    ind [max_objs], mask [max_objs])."""
    gt = gravity_center_boxes(gt_boxes.float())
    labels = gt_labels.long()
    max_objs = cfg.max_objs * cfg.dense_reg
    grid_size = torch.tensor(cfg.grid_size)
    pc_range = torch.tensor(cfg.point_cloud_range)
    voxel_size = torch.tensor(cfg.voxel_size)
    fms = grid_size[:2] // cfg.out_size_factor
    task_boxes, task_classes = [], []
    flag = 0
    for names in cfg.tasks:
        tb, tc = [], []
        for i in range(len(names)):
            m = torch.where(labels == i + flag)
            tb.append(gt[m])
            tc.append(labels[m] + 1 - flag)
        task_boxes.append(torch.cat(tb, 0))
        task_classes.append(torch.cat(tc).long())
        flag += len(names)
    heatmaps, anno_boxes, inds, masks = [], [], [], []
    for idx, names in enumerate(cfg.tasks):
        heatmap = gt.new_zeros((len(names), int(fms[1]), int(fms[0])))
        anno_box = gt.new_zeros((max_objs, 10), dtype=torch.float32)
        ind = labels.new_zeros((max_objs,), dtype=torch.int64)
        mask = gt.new_zeros((max_objs,), dtype=torch.uint8)
        num_objs = min(task_boxes[idx].shape[0], max_objs)
        for k in range(num_objs):
            cls_id = task_classes[idx][k] - 1
            width = task_boxes[idx][k][3]
            length = task_boxes[idx][k][4]
            width = width / voxel_size[0] / cfg.out_size_factor
            length = length / voxel_size[1] / cfg.out_size_factor
            if width > 0 and length > 0:
                radius = gaussian_radius((length, width), min_overlap=cfg.gaussian_overlap)
                radius = max(cfg.min_radius, int(radius))
                x, y, z = task_boxes[idx][k][0], task_boxes[idx][k][1], task_boxes[idx][k][2]
                coor_x = (x - pc_range[0]) / voxel_size[0] / cfg.out_size_factor
                coor_y = (y - pc_range[1]) / voxel_size[1] / cfg.out_size_factor
                center = torch.tensor([coor_x, coor_y], dtype=torch.float32)
                center_int = center.to(torch.int32)
                if not (0 <= center_int[0] < fms[0] and 0 <= center_int[1] < fms[1]):
                    continue
                draw_heatmap_gaussian(heatmap[cls_id], center_int, radius)
                cx, cy = center_int[0], center_int[1]
                ind[k] = cy * fms[0] + cx
                mask[k] = 1
                vx, vy = task_boxes[idx][k][7:]
                rot = task_boxes[idx][k][6]
                box_dim = task_boxes[idx][k][3:6]
                if cfg.norm_bbox:
                    box_dim = box_dim.log()
                anno_box[k] = torch.cat([center - torch.tensor([cx, cy]), z.unsqueeze(0), box_dim,
                                         torch.sin(rot).unsqueeze(0), torch.cos(rot).unsqueeze(0),
                                         vx.unsqueeze(0), vy.unsqueeze(0)])
        heatmaps.append(heatmap)
        anno_boxes.append(anno_box)
        inds.append(ind)
        masks.append(mask)
    return heatmaps, anno_boxes, inds, masks


def targets(cfg: CenterCfg, gt_boxes_list, gt_labels_list):
    """Batched targets (`get_targets`): per task stacked over the batch."""
    per = [targets_single(cfg, b, l) for b, l in zip(gt_boxes_list, gt_labels_list)]
    T = len(cfg.tasks)
    return ([torch.stack([p[0][t] for p in per]) for t in range(T)],
            [torch.stack([p[1][t] for p in per]) for t in range(T)],
            [torch.stack([p[2][t] for p in per]) for t in range(T)],
            [torch.stack([p[3][t] for p in per]) for t in range(T)])


def clamp_sigmoid(x, eps=1e-4):
    return torch.clamp(x.sigmoid(), min=eps, max=1 - eps)


def gaussian_focal_loss(pred, gaussian_target, alpha=2.0, gamma=4.0):
    eps = 1e-12
    pos_weights = gaussian_target.eq(1)
    neg_weights = (1 - gaussian_target).pow(gamma)
    pos_loss = -(pred + eps).log() * (1 - pred).pow(alpha) * pos_weights
    neg_loss = -(1 - pred + eps).log() * pred.pow(alpha) * neg_weights
    return pos_loss + neg_loss


def losses(cfg: CenterCfg, heatmap_logits, box_preds, gt_boxes_list, gt_labels_list):
    """loss_by_feat. heatmap_logits[t]: [B, ncls_t, H, W]; box_preds[t]: [B, 10, H, W] (reg, height,
    dim, rot, vel concatenated, as `preds_dict[0]['anno_box']`). Returns an ordered dict of
    task{t}.loss_heatmap / task{t}.loss_bbox."""
    hms, annos, inds, masks = targets(cfg, gt_boxes_list, gt_labels_list)
    out = {}
    for t in range(len(cfg.tasks)):
        pred_hm = clamp_sigmoid(heatmap_logits[t])
        num_pos = hms[t].eq(1).float().sum().item()
        avg = max(num_pos, 1)
        lh = gaussian_focal_loss(pred_hm, hms[t]).sum() / (avg + FLT_EPS) * cfg.loss_cls_weight
        target_box = annos[t]
        ind = inds[t]
        num = masks[t].float().sum()
        B, C = box_preds[t].shape[0], box_preds[t].shape[1]
        pred = box_preds[t].permute(0, 2, 3, 1).contiguous().view(B, -1, C)
        pred = pred.gather(1, ind.unsqueeze(2).expand(B, ind.shape[1], C))
        mask = masks[t].unsqueeze(2).expand_as(target_box).float()
        isnotnan = (~torch.isnan(target_box)).float()
        mask = mask * isnotnan
        bbox_weights = mask * mask.new_tensor(cfg.code_weights)
        l1 = torch.abs(pred - target_box) * bbox_weights
        lb = cfg.loss_bbox_weight * (l1.sum() / ((num + 1e-4) + FLT_EPS))
        out[f"task{t}.loss_heatmap"] = lh
        out[f"task{t}.loss_bbox"] = lb
    return out
