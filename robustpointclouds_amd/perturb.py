"""Autograd wrappers around the perturber / VFE kernels (SURVEY.md §8(a) rows a2–a5).

* `PerturberFn`      — VoxelPerturber.forward on a compacted [N, F] point set
                       (models/adversarial/voxel_perturber.py:120-321).
* `PerturbVoxelsFn`  — the fused hot path of AdversarialVoxelNet.extract_feat
                       (models/detectors/adversarial_voxelnet.py:85-137): valid-slot mask,
                       perturber, masked scatter back into the voxels and HardSimpleVFE, one
                       kernel sequence with no host synchronisation.
* `VoxelMeanFn`      — HardSimpleVFE alone (unperturbed path).

Parameter gradients come back already passed through the reference's grad hook
(`clamp(nan_to_num(g), -0.1, 0.1)`, voxel_perturber.py:465-475), which the kernel applies
to the full gradient of each parameter — the same value the hook sees, because each
perturber parameter is used exactly once in the graph.
"""
from __future__ import annotations

import ctypes as C

import torch

from . import _ffi
from . import stage_timer


def make_cfg(F, hidden, use_attention, training, sensor_error_bound, bn_eps=1e-3, bn_momentum=0.1,
             vfe_features=4, wgrad_split_bf16=False, act16=0):
    cfg = _ffi.PerturberCfg()
    cfg.F = int(F)
    for k in range(3):
        cfg.hidden[k] = int(hidden[k])
    cfg.use_attention = int(bool(use_attention))
    cfg.training = int(bool(training))
    cfg.sensor_error_bound = float(sensor_error_bound)
    cfg.bn_eps = float(bn_eps)
    cfg.bn_momentum = float(bn_momentum)
    cfg.vfe_features = int(vfe_features)
    cfg.wgrad_split_bf16 = int(bool(wgrad_split_bf16))
    cfg.act16 = int(act16) & 3
    return cfg


def _ptr_array(tensors):
    arr = (C.c_void_p * _ffi.PERTURBER_NPARAMS)()
    for k, t in enumerate(tensors):
        arr[k] = None if t is None else t.data_ptr()
    return arr


def _run_forward(cfg, params, x, rows, slots, num_points, out, vfe):
    if not x.is_cuda:
        raise RuntimeError("VoxelPerturber runs on the HIP kernels only: its input is a CPU tensor "
                           f"({tuple(x.shape)}); move the model and points to a ROCm device")
    lib = _ffi.load()
    dev = x.device
    wsb = lib.rpc_perturber_workspace_size(C.byref(cfg), rows, slots)
    if wsb == 0:
        raise RuntimeError("rpc_perturber_workspace_size: unsupported configuration "
                           f"F={cfg.F} hidden={list(cfg.hidden)}")
    ws = _ffi.workspace(wsb, dev)
    losses = torch.empty(8, dtype=torch.float32, device=dev)
    rc = lib.rpc_perturber_forward(C.byref(cfg), _ptr_array(params), _ffi.ptr(x), rows, slots,
                                   _ffi.ptr(num_points), _ffi.ptr(out), _ffi.ptr(vfe), _ffi.ptr(losses),
                                   _ffi.ptr(ws), wsb, _ffi.stream_of(x))
    _ffi.check(rc, "rpc_perturber_forward")
    return ws, losses


def _run_backward(cfg, params, x, rows, slots, num_points, dout, dl, ws):
    lib = _ffi.load()
    grads = [None] * _ffi.PERTURBER_NPARAMS
    for k, p in enumerate(params):
        if p is None or k in _RUNNING:
            continue
        grads[k] = torch.empty_like(p)
    rc = lib.rpc_perturber_backward(C.byref(cfg), _ptr_array(params), _ffi.ptr(x), rows, slots,
                                    _ffi.ptr(num_points), _ffi.ptr(dout), _ffi.ptr(dl), _ptr_array(grads),
                                    _ffi.ptr(ws), ws.numel(), _ffi.stream_of(x))
    _ffi.check(rc, "rpc_perturber_backward")
    return grads


_RUNNING = {6 * l + 4 for l in range(5)} | {6 * l + 5 for l in range(5)}


def _loss_grads(dl, dev):
    if dl is None:
        return torch.zeros(4, dtype=torch.float32, device=dev)
    return dl.to(torch.float32).contiguous()


class PerturberFn(torch.autograd.Function):
    """x [N, F] -> out [N, F], lvec [4] = (l2, intensity, bias, imbalance), flags [8]."""

    @staticmethod
    def forward(ctx, x, cfg, *params):
        x = x.contiguous()
        N, F = x.shape
        out = torch.empty_like(x)
        ws, losses = _run_forward(cfg, params, x, N, 1, None, out, None)
        ctx.cfg = cfg
        ctx.save_for_backward(x, ws, *[p for p in params])
        ctx.mark_non_differentiable(losses)
        ctx.set_materialize_grads(False)   # the flags' gradient stays None (no zero-fill launch)
        return out, losses[:4].clone(), losses

    @staticmethod
    def backward(ctx, dout, dlvec, _dflags):
        x, ws, *params = ctx.saved_tensors
        if not ctx.cfg.training:
            raise RuntimeError("VoxelPerturber backward is only defined in train mode")
        dev = x.device
        dout = torch.zeros_like(x) if dout is None else dout.contiguous()
        dl = _loss_grads(dlvec, dev)
        grads = _run_backward(ctx.cfg, params, x, x.shape[0], 1, None, dout, dl, ws)
        return (None, None, *grads)


class PerturbVoxelsFn(torch.autograd.Function):
    """voxels [V, P, F], num_points [V] -> vfe [V, vf], lvec [4] = (l2, intensity, bias,
    imbalance), perturbed voxels [V, P, F] (not differentiable), flags [8]
    (losses[4] = n_valid, losses[5] = NaN/empty fallback)."""

    @staticmethod
    def forward(ctx, voxels, num_points, cfg, *params):
        voxels = voxels.contiguous()
        num_points = num_points.to(torch.int32).contiguous()
        V, P, F = voxels.shape
        out = torch.empty_like(voxels)
        vfe = torch.empty((V, cfg.vfe_features), dtype=torch.float32, device=voxels.device)
        tm = stage_timer.active()
        e0 = stage_timer.TIMER.start() if tm else None
        ws, losses = _run_forward(cfg, params, voxels, V, P, num_points, out, vfe)
        if tm:
            stage_timer.TIMER.stop("perturber_fwd", e0, 2 * V * P * F * 4 + V * 4 + V * cfg.vfe_features * 4)
        ctx.cfg = cfg
        ctx.save_for_backward(voxels, num_points, ws, *params)
        ctx.mark_non_differentiable(out, losses)
        ctx.set_materialize_grads(False)   # no zero-filled [V, P, F] / flags gradients per step
        return vfe, losses[:4].clone(), out, losses

    @staticmethod
    def backward(ctx, dvfe, dlvec, _dout, _dflags):
        voxels, num_points, ws, *params = ctx.saved_tensors
        V, P, F = voxels.shape
        dev = voxels.device
        dvfe = torch.zeros((V, ctx.cfg.vfe_features), device=dev) if dvfe is None else dvfe.contiguous()
        dl = _loss_grads(dlvec, dev)
        tm = stage_timer.active()
        e0 = stage_timer.TIMER.start() if tm else None
        grads = _run_backward(ctx.cfg, params, voxels, V, P, num_points, dvfe, dl, ws)
        if tm:
            stage_timer.TIMER.stop("perturber_bwd", e0, V * P * F * 4 + V * 4 + V * ctx.cfg.vfe_features * 4)
        return (None, None, None, *grads)


class VoxelMeanFn(torch.autograd.Function):
    """HardSimpleVFE: voxels [V, P, F], num_points [V] -> [V, vf]."""

    @staticmethod
    def forward(ctx, voxels, num_points, vf):
        lib = _ffi.load()
        voxels = voxels.contiguous()
        num_points = num_points.to(torch.int32).contiguous()
        V, P, F = voxels.shape
        out = torch.empty((V, vf), dtype=torch.float32, device=voxels.device)
        _ffi.check(lib.rpc_vfe_mean_forward(_ffi.ptr(voxels), _ffi.ptr(num_points), V, P, F, vf,
                                            _ffi.ptr(out), _ffi.stream_of(voxels)), "rpc_vfe_mean_forward")
        ctx.save_for_backward(num_points)
        ctx.shape = (V, P, F, vf)
        return out

    @staticmethod
    def backward(ctx, dout):
        lib = _ffi.load()
        (num_points,) = ctx.saved_tensors
        V, P, F, vf = ctx.shape
        dvox = torch.empty((V, P, F), dtype=torch.float32, device=dout.device)
        dout = dout.contiguous()
        _ffi.check(lib.rpc_vfe_mean_backward(_ffi.ptr(dout), _ffi.ptr(num_points), V, P, F, vf,
                                             _ffi.ptr(dvox), _ffi.stream_of(dout)), "rpc_vfe_mean_backward")
        return dvox, None, None
