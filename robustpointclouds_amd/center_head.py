"""CenterHead training targets and losses on the HIP kernels.

Mirrors upstream mmdet3d `CenterHead.loss_by_feat` (targets from `get_targets_single`,
GaussianFocalLoss on clamp_sigmoid heatmaps, L1Loss on the boxes gathered at the GT centres) as
configured by the nuScenes base of configs/adversarial/adversarial-centerpoint_voxel-nuscenes.py:11-13
and called at models/detectors/adversarial_centerpoint.py:224. The whole loss (targets included) is
one autograd node over csrc/center_head.hip: heatmap logits [cells, hm_pitch] and boxes
[cells, box_pitch] in, the 2 * ntasks losses out; no host synchronisation (num_pos, the box count
and both normalisers stay on the device).
"""
from __future__ import annotations

import ctypes as C

import torch

from . import _ffi

NUS_TASKS = (("car",), ("truck", "construction_vehicle"), ("bus", "trailer"), ("barrier",),
             ("motorcycle", "bicycle"), ("pedestrian", "traffic_cone"))

# train_cfg.pts of centerpoint_voxel01_second_secfpn_head-dcn (nuScenes)
NUS_TRAIN_CFG = dict(grid_size=[1024, 1024, 40], voxel_size=[0.1, 0.1, 0.2], out_size_factor=8, dense_reg=1,
                     gaussian_overlap=0.1, max_objs=500, min_radius=2,
                     code_weights=[1.0, 1.0, 1.0, 1.0, 1.0, 1.0, 1.0, 1.0, 0.2, 0.2],
                     point_cloud_range=[-51.2, -51.2, -5.0, 51.2, 51.2, 3.0])


def center_cfg(tasks, train_cfg, B, H, W, hm_pitch, box_pitch, norm_bbox=True, loss_cls_weight=1.0,
               loss_bbox_weight=0.25) -> _ffi.RpcCenterCfg:
    if len(tasks) > 8:
        raise ValueError("at most 8 CenterHead tasks")
    c = _ffi.RpcCenterCfg()
    c.B, c.H, c.W = B, H, W
    c.ntasks = len(tasks)
    c.ncls_total = sum(len(t) for t in tasks)
    for i, t in enumerate(tasks):
        c.task_ncls[i] = len(t)
    c.max_objs = int(train_cfg["max_objs"]) * int(train_cfg.get("dense_reg", 1))
    c.min_radius = int(train_cfg["min_radius"])
    c.out_size_factor = int(train_cfg["out_size_factor"])
    c.norm_bbox = int(bool(norm_bbox))
    vs, pr = train_cfg["voxel_size"], train_cfg["point_cloud_range"]
    c.voxel_x, c.voxel_y, c.pc_x, c.pc_y = float(vs[0]), float(vs[1]), float(pr[0]), float(pr[1])
    c.gaussian_overlap = float(train_cfg["gaussian_overlap"])
    cw = train_cfg.get("code_weights") or [1.0] * 10
    for i in range(10):
        c.code_weights[i] = float(cw[i])
    c.loss_cls_weight, c.loss_bbox_weight = float(loss_cls_weight), float(loss_bbox_weight)
    c.hm_pitch, c.box_pitch = hm_pitch, box_pitch
    return c


def pack_gt(gt_boxes_list, gt_labels_list, device):
    """Per-frame [n, 9] LiDAR boxes / [n] labels -> padded device tensors [B, M, 9] fp32 and [B, M]
    int64 (-1 padding), built on the host in pinned memory and uploaded without a stream drain."""
    B = len(gt_boxes_list)
    M = max([int(b.shape[0]) for b in gt_boxes_list] + [1])
    boxes = torch.zeros((B, M, 9), dtype=torch.float32, pin_memory=torch.cuda.is_available())
    labels = torch.full((B, M), -1, dtype=torch.int64, pin_memory=torch.cuda.is_available())
    for i, (b, l) in enumerate(zip(gt_boxes_list, gt_labels_list)):
        n = int(b.shape[0])
        if n:
            boxes[i, :n] = b.detach().to("cpu", torch.float32)[:, :9]
            labels[i, :n] = l.detach().to("cpu", torch.int64)
    return boxes.to(device, non_blocking=True), labels.to(device, non_blocking=True)


class CenterLossFn(torch.autograd.Function):
    """(hm [cells, hm_pitch], box [cells, box_pitch]) -> losses [2 * ntasks] (heatmap, bbox per task)."""

    @staticmethod
    def forward(ctx, hm, box, gt_boxes, gt_labels, cfg):
        lib = _ffi.load()
        hm = hm.float().contiguous()
        box = box.float().contiguous()
        cells = cfg.B * cfg.H * cfg.W
        if hm.numel() != cells * cfg.hm_pitch or box.numel() != cells * cfg.box_pitch:
            raise ValueError("CenterLossFn: head output sizes do not match the config")
        maxg = int(gt_labels.shape[1])
        wsz = lib.rpc_center_head_workspace_size(C.byref(cfg), maxg)
        if wsz == 0:
            raise ValueError("CenterLossFn: invalid RpcCenterCfg")
        ws = _ffi.workspace(wsz, hm.device)
        out = torch.empty(2 * cfg.ntasks, dtype=torch.float32, device=hm.device)
        _ffi.check(lib.rpc_center_head_loss_forward(C.byref(cfg), _ffi.ptr(gt_boxes), _ffi.ptr(gt_labels), maxg,
                                                    _ffi.ptr(hm), _ffi.ptr(box), _ffi.ptr(out), _ffi.ptr(ws), wsz,
                                                    _ffi.stream_of(hm)), "rpc_center_head_loss_forward")
        ctx.save_for_backward(hm, box)
        ctx.ws, ctx.wsz, ctx.cfg = ws, wsz, cfg
        return out

    @staticmethod
    def backward(ctx, gl):
        lib = _ffi.load()
        hm, box = ctx.saved_tensors
        gl = gl.float().contiguous()
        dhm = torch.empty_like(hm)
        dbox = torch.empty_like(box)
        _ffi.check(lib.rpc_center_head_loss_backward(C.byref(ctx.cfg), _ffi.ptr(hm), _ffi.ptr(box), _ffi.ptr(gl),
                                                     _ffi.ptr(dhm), _ffi.ptr(dbox), _ffi.ptr(ctx.ws), ctx.wsz,
                                                     _ffi.stream_of(hm)), "rpc_center_head_loss_backward")
        ctx.ws = None
        return dhm, dbox, None, None, None


def center_targets(cfg, ws, maxg):
    """Views of the targets kept in a forward workspace: heatmap [B, H, W, ncls], ind / mask
    [B, T, max_objs], anno [B, T, max_objs, 10] (device tensors sharing the workspace)."""
    lib = _ffi.load()
    ptrs = [C.c_void_p() for _ in range(4)]
    _ffi.check(lib.rpc_center_head_targets(C.byref(cfg), maxg, _ffi.ptr(ws), *[C.byref(p) for p in ptrs]),
               "rpc_center_head_targets")
    base = ws.data_ptr()
    B, H, W, T, MO, N = cfg.B, cfg.H, cfg.W, cfg.ntasks, cfg.max_objs, cfg.ncls_total

    def view(p, dtype, shape):
        off = p.value - base
        n = 1
        for s in shape:
            n *= s
        esz = torch.tensor([], dtype=dtype).element_size()
        return ws[off:off + n * esz].view(dtype).view(*shape)

    return (view(ptrs[0], torch.float32, (B, H, W, N)), view(ptrs[1], torch.int32, (B, T, MO)),
            view(ptrs[2], torch.int32, (B, T, MO)), view(ptrs[3], torch.float32, (B, T, MO, 10)))
