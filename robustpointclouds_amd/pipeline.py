"""Training data pipeline on the GPU.

configs/_base_/kitti-3d-car.py:42-68 (the 3-class config inherits the same transforms):
LoadPointsFromFile(load_dim=4, use_dim=4) -> ... -> RandomFlip3D(0.5) -> GlobalRotScaleTrans(
rot_range ±pi/4, scale 0.95-1.05) -> PointsRangeFilter -> ObjectRangeFilter -> PointShuffle.

* `load_points_from_file` — the KITTI / mmdet3d `.bin` format: float32 records of `load_dim`
  values, the first `use_dim` kept (host file read; the frames then go to HBM once).
* `GpuTrainAugment` — the per-frame random transforms for a whole batch in two HIP launches
  (csrc/augment.hip: `rpc_augment_points`, `rpc_augment_boxes`). The random draws are made on the
  host in the order upstream mmdet3d makes them per frame (RandomFlip3D: np.random.rand for the
  horizontal then the vertical flip; GlobalRotScaleTrans: np.random.uniform rotation, uniform scale,
  np.random.normal translation), so a seeded numpy RNG reproduces the reference's parameters; the
  arithmetic, the range filters, the compaction and the shuffle run on the device with no host
  read of the surviving point counts (dropped rows are NaN, which the voxeliser rejects; dropped
  boxes become label -1 padding).
  PointShuffle: upstream permutes with torch.randperm on the host RNG; here `shuffle="device"` is a
  seeded uniform permutation per frame computed on the GPU (same distribution, different stream).
* ObjectSample (GT-database paste) and ObjectNoise need the KITTI info / db pickles and per-object
  collision tests; they are not part of the GPU pipeline (no dataset in this build's scope).
"""
from __future__ import annotations

import ctypes as C
from typing import List, Optional, Sequence

import numpy as np
import torch

from . import _ffi

AUG_DTYPE = np.dtype([("flip_h", "<i4"), ("flip_v", "<i4"), ("rot", "<f4"), ("cosr", "<f4"), ("sinr", "<f4"),
                      ("scale", "<f4"), ("tx", "<f4"), ("ty", "<f4"), ("tz", "<f4")])


def load_points_from_file(path: str, load_dim: int = 4, use_dim=4) -> np.ndarray:
    """mmdet3d LoadPointsFromFile for `.bin` point files: [N, load_dim] float32 -> the use_dim columns."""
    pts = np.fromfile(path, dtype=np.float32)
    if pts.size % load_dim:
        raise ValueError(f"{path}: {pts.size} floats is not a multiple of load_dim={load_dim}")
    pts = pts.reshape(-1, load_dim)
    cols = list(range(use_dim)) if isinstance(use_dim, int) else list(use_dim)
    return np.ascontiguousarray(pts[:, cols])


class GpuTrainAugment:
    def __init__(self, point_cloud_range: Sequence[float], flip_ratio_bev_horizontal=0.5,
                 flip_ratio_bev_vertical=0.0, rot_range=(-0.78539816, 0.78539816), scale_ratio_range=(0.95, 1.05),
                 translation_std=(0.0, 0.0, 0.0), shuffle: Optional[str] = "device"):
        self.pc_range = [float(v) for v in point_cloud_range]
        self.flip_h, self.flip_v = float(flip_ratio_bev_horizontal), float(flip_ratio_bev_vertical)
        self.rot_range = [float(v) for v in rot_range]
        self.scale_range = [float(v) for v in scale_ratio_range]
        self.translation_std = [float(v) for v in translation_std]
        if shuffle not in (None, "device"):
            raise ValueError("shuffle must be None or 'device'")
        self.shuffle = shuffle

    def sample(self, batch: int, rng=np.random) -> np.ndarray:
        """Per-frame random parameters, drawn in the upstream order (RandomFlip3D then
        GlobalRotScaleTrans, frame after frame); cos / sin formed like torch (float32)."""
        fr = np.zeros(batch, AUG_DTYPE)
        for b in range(batch):
            fr[b]["flip_h"] = int(rng.rand() < self.flip_h)
            fr[b]["flip_v"] = int(rng.rand() < self.flip_v)
            rot = rng.uniform(self.rot_range[0], self.rot_range[1])
            scale = rng.uniform(self.scale_range[0], self.scale_range[1])
            trans = rng.normal(scale=self.translation_std, size=3).T
            ang = torch.tensor(rot, dtype=torch.float32)
            fr[b]["rot"] = np.float32(rot)
            fr[b]["cosr"] = float(torch.cos(ang))
            fr[b]["sinr"] = float(torch.sin(ang))
            fr[b]["scale"] = np.float32(scale)
            fr[b]["tx"], fr[b]["ty"], fr[b]["tz"] = (np.float32(t) for t in trans)
        return fr

    def __call__(self, points: torch.Tensor, offsets: torch.Tensor, gt_boxes: Optional[torch.Tensor] = None,
                 gt_labels: Optional[torch.Tensor] = None, frames: Optional[np.ndarray] = None, seed: int = 0,
                 rng=np.random):
        """points [P, F] (frames concatenated, cuda), offsets [B+1] int32 (cuda) -> (points', offsets',
        boxes', labels'). Boxes / labels ([B, M, 7] / [B, M] int64, -1 padding) are updated in place."""
        lib = _ffi.load()
        if not points.is_cuda:
            raise RuntimeError("GpuTrainAugment runs on the HIP kernels only (no CPU path)")
        points = points.float().contiguous()
        offsets = offsets.to(device=points.device, dtype=torch.int32).contiguous()
        B = offsets.numel() - 1
        P, F = points.shape
        if frames is None:
            frames = self.sample(B, rng)
        fr = torch.from_numpy(np.ascontiguousarray(frames).view(np.uint8)).pin_memory().to(points.device,
                                                                                            non_blocking=True)
        out = torch.empty_like(points)
        out_off = torch.empty(B + 1, dtype=torch.int32, device=points.device)
        wsz = lib.rpc_augment_points_workspace_size(F, P)
        ws = _ffi.workspace(wsz, points.device)
        st = _ffi.stream_of(points)
        rg = _ffi.float_arr(self.pc_range)
        _ffi.check(lib.rpc_augment_points(_ffi.ptr(points), F, P, _ffi.ptr(offsets), B, _ffi.ptr(fr), rg,
                                          1 if self.shuffle else 0, C.c_ulonglong(seed & (2 ** 64 - 1)),
                                          _ffi.ptr(out), _ffi.ptr(out_off), _ffi.ptr(ws), wsz, st),
                   "rpc_augment_points")
        if gt_boxes is not None:
            if gt_labels is None or gt_labels.dtype != torch.int64 or gt_boxes.dtype != torch.float32:
                raise TypeError("gt_boxes float32 [B, M, 7] and gt_labels int64 [B, M] expected")
            _ffi.check(lib.rpc_augment_boxes(_ffi.ptr(gt_boxes), _ffi.ptr(gt_labels), B, gt_boxes.shape[1],
                                             _ffi.ptr(fr), rg, st), "rpc_augment_boxes")
        return out, out_off, gt_boxes, gt_labels


def concat_frames(frames: List[np.ndarray], device) -> (torch.Tensor, torch.Tensor):
    """Host frames -> one [P, F] device tensor + [B+1] int32 device offsets (pinned, non-blocking)."""
    off = np.zeros(len(frames) + 1, np.int32)
    off[1:] = np.cumsum([f.shape[0] for f in frames])
    pts = torch.from_numpy(np.concatenate(frames, 0).astype(np.float32)).pin_memory().to(device, non_blocking=True)
    return pts, torch.from_numpy(off).pin_memory().to(device, non_blocking=True)
