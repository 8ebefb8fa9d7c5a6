"""PARITY ORACLE — TEST INFRASTRUCTURE ONLY (tests/).

CPU restatement (torch float32) of the per-frame training transforms of
configs/_base_/kitti-3d-car.py:42-68, upstream mmdet3d v1.x semantics (not vendored here, so
parity w.r.t. upstream is unpinned; the rotation is written as the two products and sum of the
2x2 block of rot_mat_T rather than a BLAS matmul, which can differ from it by one ulp):
  RandomFlip3D        points / boxes y -> -y, yaw -> -yaw (horizontal); x -> -x, yaw -> pi - yaw (vertical)
  GlobalRotScaleTrans rotate about z (rot_mat_T = [[c, s, 0], [-s, c, 0], [0, 0, 1]]), yaw += angle,
                      scale xyz (boxes: centre and dims), translate
  PointsRangeFilter   strict in_range_3d;  ObjectRangeFilter strict in_range_bev + limit_yaw(0.5, 2 pi)
"""
from __future__ import annotations

import numpy as np
import torch


def augment_frame(points: torch.Tensor, boxes: torch.Tensor, labels: torch.Tensor, fr, pc_range):
    """points [N, F] float32, boxes [M, 7], labels [M] (-1 = padding); fr: one AUG_DTYPE record.
    Returns (kept points in order, boxes, labels) with dropped boxes as padding (label -1, unit size)."""
    p = points.clone().float()
    x, y, z = p[:, 0].clone(), p[:, 1].clone(), p[:, 2].clone()
    c, s = torch.tensor(float(fr["cosr"]), dtype=torch.float32), torch.tensor(float(fr["sinr"]), dtype=torch.float32)
    sc = torch.tensor(float(fr["scale"]), dtype=torch.float32)
    t = [torch.tensor(float(fr[k]), dtype=torch.float32) for k in ("tx", "ty", "tz")]
    if fr["flip_h"]:
        y = -y
    if fr["flip_v"]:
        x = -x
    x, y = x * c + y * (-s), x * s + y * c
    x, y, z = x * sc, y * sc, z * sc
    x, y, z = x + t[0], y + t[1], z + t[2]
    p[:, 0], p[:, 1], p[:, 2] = x, y, z
    r = pc_range
    keep = (x > r[0]) & (y > r[1]) & (z > r[2]) & (x < r[3]) & (y < r[4]) & (z < r[5])
    bo, la = boxes.clone().float(), labels.clone()
    for j in range(bo.shape[0]):
        if la[j] < 0:
            continue
        bx, by, bz, yaw = bo[j, 0], bo[j, 1], bo[j, 2], bo[j, 6]
        if fr["flip_h"]:
            by, yaw = -by, -yaw
        if fr["flip_v"]:
            bx, yaw = -bx, -yaw + torch.tensor(np.pi, dtype=torch.float32)
        bx, by = bx * c + by * (-s), bx * s + by * c
        yaw = yaw + torch.tensor(float(fr["rot"]), dtype=torch.float32)
        bx, by, bz = bx * sc, by * sc, bz * sc
        dims = bo[j, 3:6] * sc
        bx, by, bz = bx + t[0], by + t[1], bz + t[2]
        if not bool((bx > r[0]) & (by > r[1]) & (bx < r[3]) & (by < r[4])):
            la[j] = -1
            bo[j, 3:6] = 1.0
            continue
        period = torch.tensor(2 * np.pi, dtype=torch.float32)
        yaw = yaw - torch.floor(yaw / period + torch.tensor(0.5, dtype=torch.float32)) * period
        bo[j, 0], bo[j, 1], bo[j, 2], bo[j, 6] = bx, by, bz, yaw
        bo[j, 3:6] = dims
    return p[keep], bo, la
