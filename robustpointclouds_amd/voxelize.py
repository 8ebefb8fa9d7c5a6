"""Hard voxelisation on the GPU.

`Voxelization` mirrors mmcv.ops.Voxelization (the `voxel_layer` of upstream
Det3DDataPreprocessor, configured at
configs/adversarial/adversarial-second_hv_secfpn_8xb6-80e_kitti-3d-car.py:48-53) and
`voxelize_batch` mirrors Det3DDataPreprocessor.voxelize for voxel_type='hard': per-frame
voxelisation, batch id padded in front of (z, y, x), everything concatenated. Here all B
frames go through one kernel sequence (rpc_hard_voxelize) instead of a Python loop; one
device->host copy of the voxel count is the only synchronisation.
"""
from __future__ import annotations

from typing import Sequence

import torch
from torch import nn

from . import _ffi
from . import stage_timer


def _frame_offsets(sizes: Sequence[int], device) -> torch.Tensor:
    """[B+1] int32 prefix offsets on `device`, uploaded from pinned memory without blocking the host
    (a pageable torch.tensor(..., device=cuda) would wait for the whole stream to drain)."""
    off = [0]
    for n in sizes:
        off.append(off[-1] + int(n))
    host = torch.tensor(off, dtype=torch.int32)
    if torch.device(device).type != "cuda":
        return host
    return host.pin_memory().to(device, non_blocking=True)


def voxelize_batch(points: torch.Tensor, frame_offsets: torch.Tensor, voxel_size, point_cloud_range,
                   max_num_points: int, max_voxels: int, defer: bool = False):
    """Voxelise B concatenated frames (defer=True: return a PendingVoxels instead of reading V now).

    points:         [P, F] float32 cuda, frames back to back
    frame_offsets:  [B+1] int32 cuda
    returns voxels [V, max_num_points, F], coors [V, 4] int32 (b, z, y, x),
            num_points [V] int32, voxel_num [B+1] int32 (per frame, then total; on device)
    """
    lib = _ffi.load()
    if points.dtype != torch.float32 or points.dim() != 2:
        raise ValueError("points must be a [P, F] float32 tensor")
    points = points.contiguous()
    frame_offsets = frame_offsets.to(device=points.device, dtype=torch.int32).contiguous()
    B = frame_offsets.numel() - 1
    P, F = points.shape
    dev = points.device
    cap = B * max_voxels
    voxels = torch.empty((cap, max_num_points, F), dtype=torch.float32, device=dev)
    coors = torch.empty((cap, 4), dtype=torch.int32, device=dev)
    num_points = torch.empty((cap,), dtype=torch.int32, device=dev)
    voxel_num = torch.empty((B + 1,), dtype=torch.int32, device=dev)
    wsb = lib.rpc_hard_voxelize_workspace_size(P, B)
    ws = _ffi.workspace(wsb, dev)
    tm = stage_timer.active()
    e0 = stage_timer.TIMER.start() if tm else None
    rc = lib.rpc_hard_voxelize(_ffi.ptr(points), F, P, _ffi.ptr(frame_offsets), B,
                               _ffi.float_arr(voxel_size), _ffi.float_arr(point_cloud_range),
                               int(max_num_points), int(max_voxels), _ffi.ptr(voxels), _ffi.ptr(coors),
                               _ffi.ptr(num_points), _ffi.ptr(voxel_num), _ffi.ptr(ws), wsb,
                               _ffi.stream_of(points))
    _ffi.check(rc, "rpc_hard_voxelize")
    if tm:
        vrow = max_num_points * F * 4 + 16 + 4
        stage_timer.TIMER.stop("voxelize", e0, lambda: P * F * 4 + int(voxel_num[B]) * vrow)
    if defer:
        return PendingVoxels(voxels, coors, num_points, voxel_num, B)
    V = int(voxel_num[B].item())  # the one host sync: output shapes
    return voxels[:V], coors[:V], num_points[:V], voxel_num


class PendingVoxels:
    """A voxelisation whose kernels are queued (normally on a side stream) and whose voxel count V —
    the one host read — is copied to pinned memory behind an event instead of draining the stream.
    `result(consumer)` makes the consumer stream wait for the voxelisation, marks the outputs as used
    by it (caching-allocator safety across streams) and reads V, by then normally long complete."""

    def __init__(self, voxels, coors, num_points, voxel_num, B):
        self.t = (voxels, coors, num_points, voxel_num)
        self.host = torch.empty(1, dtype=torch.int32, pin_memory=True)
        self.host.copy_(voxel_num[B:], non_blocking=True)
        self.ev = torch.cuda.Event()
        self.ev.record(torch.cuda.current_stream(voxels.device))

    def count(self) -> int:
        """V (a host read: waits for the voxelisation kernels only)."""
        self.ev.synchronize()
        return int(self.host[0])

    def result(self, consumer=None):
        voxels, coors, num_points, voxel_num = self.t
        if consumer is not None:
            consumer.wait_event(self.ev)
            for x in self.t:
                x.record_stream(consumer)
        self.ev.synchronize()
        V = int(self.host[0])
        return voxels[:V], coors[:V], num_points[:V], voxel_num


class Voxelization(nn.Module):
    """mmcv.ops.Voxelization-compatible module (hard voxelisation, deterministic)."""

    def __init__(self, voxel_size, point_cloud_range, max_num_points, max_voxels=20000,
                 deterministic=True):
        super().__init__()
        self.voxel_size = [float(v) for v in voxel_size]
        self.point_cloud_range = [float(v) for v in point_cloud_range]
        self.max_num_points = int(max_num_points)
        self.max_voxels = max_voxels if isinstance(max_voxels, (tuple, list)) else (max_voxels, max_voxels)
        self.deterministic = deterministic

    def _cap(self):
        return int(self.max_voxels[0] if self.training else self.max_voxels[1])

    def forward(self, points: torch.Tensor):
        """One frame [N, F] -> voxels [V, P, F], coors [V, 3] (z, y, x), num_points [V]."""
        off = _frame_offsets([points.shape[0]], points.device)
        v, c, n, _ = voxelize_batch(points, off, self.voxel_size, self.point_cloud_range,
                                    self.max_num_points, self._cap())
        return v, c[:, 1:].contiguous(), n

    def voxelize_frames(self, points_list: Sequence[torch.Tensor]):
        """Det3DDataPreprocessor.voxelize (hard): list of frames -> batched voxel dict."""
        dev = points_list[0].device
        pts = torch.cat([p.contiguous() for p in points_list], 0)
        off = _frame_offsets([p.shape[0] for p in points_list], dev)
        v, c, n, vn = voxelize_batch(pts, off, self.voxel_size, self.point_cloud_range,
                                     self.max_num_points, self._cap())
        return dict(voxels=v, coors=c, num_points=n, voxel_num=vn)

    def voxelize_frames_deferred(self, points_list: Sequence[torch.Tensor]) -> PendingVoxels:
        """voxelize_frames with the kernels queued on the current stream and V read later
        (`PendingVoxels.result`); the trainer's batch prefetch runs this on a side stream."""
        dev = points_list[0].device
        pts = torch.cat([p.contiguous() for p in points_list], 0)
        off = _frame_offsets([p.shape[0] for p in points_list], dev)
        return voxelize_batch(pts, off, self.voxel_size, self.point_cloud_range, self.max_num_points,
                              self._cap(), defer=True)
