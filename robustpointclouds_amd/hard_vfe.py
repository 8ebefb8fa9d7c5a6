"""HardVFE — the per-voxel PointNet MLP + max voxel encoder on the HIP kernels (csrc/hard_vfe.hip).

Mirrors upstream mmdet3d `HardVFE` / `VFELayer` (mmdet3d/models/voxel_encoders/voxel_encoder.py, not
vendored in /root/reference): same constructor arguments, same sub-module names (`vfe_layers.<i>.linear`,
`vfe_layers.<i>.norm`) so mmdet3d state dicts load unchanged, same forward signature
`(features [V, T, F], num_points [V], coors [V, 4]) -> [V, C_last]`. It drops into the reference's
detectors wherever they call their voxel encoder (models/detectors/adversarial_voxelnet.py:135-137,
adversarial_centerpoint.py:100). Semantics: oracle/hard_vfe.py. Image fusion (`fusion_layer`) is
outside the hot path and raises.
"""
from __future__ import annotations

import ctypes as C

import torch
from torch import nn

from . import _ffi
from .registry import MODELS


class VFELayer(nn.Module):
    """Parameter holder with mmdet3d VFELayer's names (Linear without bias, BatchNorm1d); the fused
    HardVFE kernels run every layer, so it has no forward of its own."""

    def __init__(self, in_channels, out_channels, norm_cfg=None, max_out=True, cat_max=True):
        super().__init__()
        norm_cfg = dict(norm_cfg or dict(type="BN1d", eps=1e-3, momentum=0.01))
        if norm_cfg.get("type", "BN1d") not in ("BN1d", "BN"):
            raise NotImplementedError(f"VFELayer norm {norm_cfg['type']} (BN1d only)")
        self.cat_max = cat_max
        self.max_out = max_out
        self.norm = nn.BatchNorm1d(out_channels, eps=norm_cfg.get("eps", 1e-3), momentum=norm_cfg.get("momentum", 0.01))
        self.linear = nn.Linear(in_channels, out_channels, bias=False)


def _cfg(m: "HardVFE", T: int, training: bool):
    c = _ffi.RpcHardVfeCfg()
    c.F = int(m.raw_features)
    c.T = int(T)
    c.nlayers = len(m.vfe_layers)
    for i, L in enumerate(m.vfe_layers):
        c.channels[i] = int(L.linear.out_features)
    c.with_cluster_center = int(m._with_cluster_center)
    c.with_voxel_center = int(m._with_voxel_center)
    c.with_distance = int(m._with_distance)
    c.training = int(bool(training))
    for d in range(3):
        c.voxel_size[d] = float(m.voxel_size[d])
        c.pc_range_min[d] = float(m.point_cloud_range[d])
    n0 = m.vfe_layers[0].norm
    c.bn_eps = float(n0.eps)
    c.bn_momentum = float(n0.momentum)
    return c


def _ptrs(ts):
    arr = (C.c_void_p * len(ts))()
    for k, t in enumerate(ts):
        arr[k] = t.data_ptr()
    return arr


class HardVFEFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, features, num_points, coors, module, training, *weights):
        if not features.is_cuda:
            raise RuntimeError("HardVFE runs on the HIP kernels only: its input is a CPU tensor "
                               f"({tuple(features.shape)}); move the model and voxels to a ROCm device")
        lib = _ffi.load()
        V, T, F = features.shape
        if F != module.raw_features:
            raise ValueError(f"HardVFE built for {module.raw_features} point features, got {F}")
        feats = features.contiguous().float()
        npts = num_points.to(torch.int32).contiguous()
        co = coors.to(torch.int32).contiguous()
        cfg = _cfg(module, T, training)
        wsb = lib.rpc_hard_vfe_workspace_size(C.byref(cfg), V)
        if wsb == 0:
            raise RuntimeError(f"rpc_hard_vfe: unsupported configuration (F={F}, T={T}, "
                               f"channels={[L.linear.out_features for L in module.vfe_layers]}, "
                               f"decorated width {module.in_channels} > 16?)")
        ws = _ffi.workspace(wsb, features.device)
        params = []
        for L in module.vfe_layers:
            params += [L.linear.weight, L.norm.weight, L.norm.bias, L.norm.running_mean, L.norm.running_var]
        params = [p if p.is_contiguous() else p.contiguous() for p in params]
        out = torch.empty(V, cfg.channels[cfg.nlayers - 1], dtype=torch.float32, device=features.device)
        st = _ffi.stream_of(features)
        _ffi.check(lib.rpc_hard_vfe_forward(C.byref(cfg), _ptrs(params), _ffi.ptr(feats), _ffi.ptr(npts),
                                            _ffi.ptr(co), V, _ffi.ptr(out), _ffi.ptr(ws), wsb, st),
                   "rpc_hard_vfe_forward")
        if training:
            _ffi.bump_batches([L.norm for L in module.vfe_layers])
        ctx.save_for_backward(feats, npts, co, *params)
        ctx.cfg, ctx.ws, ctx.wsb, ctx.nw = cfg, ws, wsb, len(weights)
        ctx.in_dtype = features.dtype
        return out

    @staticmethod
    def backward(ctx, dout):
        lib = _ffi.load()
        feats, npts, co, *params = ctx.saved_tensors
        cfg = ctx.cfg
        if not cfg.training:
            raise RuntimeError("HardVFE backward runs in training mode only (BatchNorm batch statistics)")
        V = feats.shape[0]
        dfeat = torch.empty_like(feats)
        grads = []
        for l in range(cfg.nlayers):
            W, g, b = params[5 * l], params[5 * l + 1], params[5 * l + 2]
            grads += [torch.empty_like(W), torch.empty_like(g), torch.empty_like(b)]
        dout = dout.contiguous().float()
        _ffi.check(lib.rpc_hard_vfe_backward(C.byref(cfg), _ptrs(params), _ffi.ptr(feats), _ffi.ptr(npts),
                                             _ffi.ptr(co), V, _ffi.ptr(dout),
                                             _ffi.ptr(dfeat), _ptrs(grads), _ffi.ptr(ctx.ws), ctx.wsb,
                                             _ffi.stream_of(feats)),
                   "rpc_hard_vfe_backward")
        # the kernels compute in fp32; autograd needs the gradient in the input's dtype (bf16 / fp16 voxels)
        return (dfeat.to(ctx.in_dtype), None, None, None, None, *grads)


@MODELS.register_module()
class HardVFE(nn.Module):
    """upstream mmdet3d HardVFE (same arguments and defaults)."""

    def __init__(self, in_channels=4, feat_channels=(), with_distance=False, with_cluster_center=False,
                 with_voxel_center=False, voxel_size=(0.2, 0.2, 4), point_cloud_range=(0, -40, -3, 70.4, 40, 1),
                 norm_cfg=dict(type="BN1d", eps=1e-3, momentum=0.01), mode="max", fusion_layer=None,
                 return_point_feats=False):
        super().__init__()
        assert len(feat_channels) > 0
        if fusion_layer is not None:
            raise NotImplementedError("HardVFE fusion_layer (image fusion) is outside the hot path")
        if mode != "max":
            raise NotImplementedError(f"HardVFE mode {mode!r} (VFELayer aggregates by max)")
        self.raw_features = in_channels
        if with_cluster_center:
            in_channels += 3
        if with_voxel_center:
            in_channels += 3
        if with_distance:
            in_channels += 1
        self.in_channels = in_channels
        self._with_distance = with_distance
        self._with_cluster_center = with_cluster_center
        self._with_voxel_center = with_voxel_center
        self.return_point_feats = return_point_feats
        self.voxel_size = tuple(voxel_size)
        self.point_cloud_range = tuple(point_cloud_range)
        self.vx, self.vy, self.vz = voxel_size
        self.x_offset = self.vx / 2 + point_cloud_range[0]
        self.y_offset = self.vy / 2 + point_cloud_range[1]
        self.z_offset = self.vz / 2 + point_cloud_range[2]
        chans = [self.in_channels] + list(feat_channels)
        layers = []
        for i in range(len(chans) - 1):
            inf = chans[i] * (2 if i > 0 else 1)
            last = i == len(chans) - 2
            layers.append(VFELayer(inf, chans[i + 1], norm_cfg=norm_cfg, max_out=True, cat_max=not last))
        self.vfe_layers = nn.ModuleList(layers)
        self.num_vfe = len(layers)
        self.fusion_layer = None

    def forward(self, features, num_points, coors, img_feats=None, img_metas=None, *args, **kwargs):
        ws = []
        for L in self.vfe_layers:
            ws += [L.linear.weight, L.norm.weight, L.norm.bias]
        return HardVFEFn.apply(features, num_points, coors, self, self.training, *ws)
