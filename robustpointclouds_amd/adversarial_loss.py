"""Loss combination of AdversarialVoxelNet.loss, device-side.

Restates models/detectors/adversarial_voxelnet.py:187-427 without its host
synchronisations (`.item()` at :229 and :405): the data-dependent branches become
`torch.where` on device scalars, with identical values and gradients:
  det_loss_total = clamp(sum clamp(v, 0, 100) over Tensor-valued 'loss' keys, skipping
                   NaN/Inf, 0, 500)                                          (:203-215)
  loss_adversarial = clamp(-det - 10 (l2 - 0.05), -10, 10) if det > 0 else 0  (:281-300, :366-367)
  loss_intensity = 3 I, loss_bias = 10 B, loss_imbalance = 10 S               (:378-391)
  loss_adversarial += 0.01 (loss_intensity + loss_bias + loss_imbalance)     (:395-398)
  reg_scale = max(0.1, 1 - (epoch+1)/30) x {0.01 | 0.1 | 0.3 | 1} by l2        (:401-411)
  loss_l2_regularization = regularization_weight * reg_scale * l2            (:413)
  perturbation_l2_norm = l2.detach()                                         (:421)
With upstream's list-valued head losses (Anchor3DHead), det is identically 0, so
loss_adversarial = 0.01 * aux (SURVEY.md finding 3).
"""
from __future__ import annotations

import torch

from . import _ffi

_TAIL_KEYS = ("loss_cls", "loss_bbox", "loss_dir", "loss_adversarial", "loss_intensity", "loss_bias",
              "loss_imbalance", "loss_l2_regularization", "perturbation_l2_norm")


class FusedLosses(dict):
    """Loss dict whose entries are views of one device vector; `.total` is parse_losses' sum."""
    total = None


class LossTailFn(torch.autograd.Function):
    """(head [3], perturber [4]) -> out [10] (csrc/step_tail.hip, rpc_loss_tail_forward/backward)."""

    @staticmethod
    def forward(ctx, head3, pert4, reg_coef):
        lib = _ffi.load()
        head3, pert4 = head3.detach().float().contiguous(), pert4.detach().float().contiguous()
        out = torch.empty(10, dtype=torch.float32, device=head3.device)
        _ffi.check(lib.rpc_loss_tail_forward(_ffi.ptr(head3), _ffi.ptr(pert4), float(reg_coef), _ffi.ptr(out),
                                             _ffi.stream_of(out)), "rpc_loss_tail_forward")
        ctx.save_for_backward(pert4)
        ctx.reg_coef = float(reg_coef)
        return out

    @staticmethod
    def backward(ctx, g):
        lib = _ffi.load()
        (pert4,) = ctx.saved_tensors
        g = g.float().contiguous()
        gh = torch.empty(3, dtype=torch.float32, device=g.device)
        gp = torch.empty(4, dtype=torch.float32, device=g.device)
        _ffi.check(lib.rpc_loss_tail_backward(_ffi.ptr(pert4), ctx.reg_coef, _ffi.ptr(g), _ffi.ptr(gh), _ffi.ptr(gp),
                                              _ffi.stream_of(g)), "rpc_loss_tail_backward")
        return gh, gp, None


def _fused_tail(losses_pts, loss_dict, epoch, regularization_weight):
    """The HIP tail when the head losses are upstream's lists (det_loss_total = 0) of one packed
    [cls, bbox, dir] vector and the perturber losses one packed [4] vector, all on the GPU."""
    head3 = getattr(losses_pts, "packed", None)
    pert4 = getattr(loss_dict, "packed", None)
    if head3 is None or pert4 is None or not head3.is_cuda or set(losses_pts) != {"loss_cls", "loss_bbox", "loss_dir"}:
        return None
    reg_scale = max(0.1, 1.0 - ((epoch + 1) / 30.0))
    out = LossTailFn.apply(head3, pert4, float(regularization_weight * reg_scale))
    res = FusedLosses()
    for i, k in enumerate(_TAIL_KEYS):
        v = out[i]
        res[k] = [v] if i < 3 else (v.detach() if k == "perturbation_l2_norm" else v)
    res.total = out[9]
    return res


class CenterTailFn(torch.autograd.Function):
    """(task losses [n], l2 []) -> out [n + 4] (csrc/step_tail.hip, rpc_center_tail_forward/backward): the
    AdversarialCenterPoint combination + parse_losses in one single-lane kernel each way."""

    @staticmethod
    def forward(ctx, v, l2, negw, rw):
        lib = _ffi.load()
        v = v.detach().float().contiguous()
        l2c = l2.detach().float().reshape(1).contiguous()
        n = v.numel()
        out = torch.empty(n + 4, dtype=torch.float32, device=v.device)
        _ffi.check(lib.rpc_center_tail_forward(_ffi.ptr(v), n, _ffi.ptr(l2c), float(negw), float(rw), _ffi.ptr(out),
                                               _ffi.stream_of(out)), "rpc_center_tail_forward")
        ctx.save_for_backward(v)
        ctx.negw, ctx.rw, ctx.l2_shape = float(negw), float(rw), l2.shape
        return out

    @staticmethod
    def backward(ctx, g):
        lib = _ffi.load()
        (v,) = ctx.saved_tensors
        g = g.float().contiguous()
        gv = torch.empty_like(v)
        gl2 = torch.empty(1, dtype=torch.float32, device=g.device)
        _ffi.check(lib.rpc_center_tail_backward(_ffi.ptr(v), v.numel(), ctx.negw, ctx.rw, _ffi.ptr(g), _ffi.ptr(gv),
                                                _ffi.ptr(gl2), _ffi.stream_of(g)), "rpc_center_tail_backward")
        return gv, gl2.reshape(ctx.l2_shape), None, None


def center_combination(losses: dict, l2, w: float, regularization_weight: float, device) -> dict:
    """AdversarialCenterPoint.loss_by_feat_single's combination in torch ops
    (models/detectors/adversarial_centerpoint.py:203-257, with the l2 scalar of the documented :81 fix): every
    Tensor-valued 'loss' entry clamped to [0, 100] and NaN/Inf-skipped, summed; loss_adversarial = -w * det when
    det > 0 (the `.item() > 0` branch of :232 as a device select); loss_l2_regularization = regularization_weight
    * l2; perturbation_l2_norm. fused_center_tail computes the same values on the HIP tail."""
    losses = dict(losses)
    det = torch.zeros((), device=device)
    for k, v in losses.items():
        if "loss" in k and isinstance(v, torch.Tensor):
            c = torch.clamp(v, min=0.0, max=100.0)
            det = det + torch.where(torch.isfinite(c), c, torch.zeros_like(c))
    adv = -w * det
    losses["loss_adversarial"] = torch.where(det > 0, adv, torch.zeros_like(adv))
    losses["loss_l2_regularization"] = regularization_weight * l2
    losses["perturbation_l2_norm"] = l2.detach()
    return losses


def fused_center_tail(task_losses: dict, packed, l2, w: float, regularization_weight: float):
    """AdversarialCenterPoint.loss_by_feat_single's combination over the CenterHead's packed task losses (a
    PackedCenterLosses dict whose values are packed[0..n) in order): a FusedLosses dict (views of one device
    vector) whose `.total` is parse_losses' sum, or None when the inputs are not that layout (or more task losses
    than rpc_center_tail_forward's one-wave-per-256 kernel takes)."""
    n = len(task_losses)
    if (n > 256 or packed is None or not packed.is_cuda or packed.dim() != 1 or packed.numel() != n or not isinstance(l2, torch.Tensor)
            or not l2.is_cuda or l2.numel() != 1 or packed.dtype != torch.float32 or l2.dtype != torch.float32):
        return None
    out = CenterTailFn.apply(packed, l2, -w, regularization_weight)
    res = FusedLosses()
    for i, k in enumerate(task_losses):
        res[k] = out[i]
    res["loss_adversarial"] = out[n]
    res["loss_l2_regularization"] = out[n + 1]
    res["perturbation_l2_norm"] = out[n + 2].detach()
    res.total = out[n + 3]
    return res


def _zero(device):
    return torch.tensor(0.0, device=device, requires_grad=True)


def combine_adversarial_losses(losses_pts: dict, l2, loss_dict, epoch: int, regularization_weight: float,
                               training: bool, device) -> dict:
    losses = dict(losses_pts)
    if not training or l2 is None:                                          # :422-425
        losses["loss_adversarial"] = _zero(device)
        losses["loss_l2_regularization"] = _zero(device)
        return losses
    fused = _fused_tail(losses_pts, loss_dict, epoch, regularization_weight) if loss_dict is not None else None
    if fused is not None:
        return fused
    tensor_items = [v for k, v in losses_pts.items() if "loss" in k and isinstance(v, torch.Tensor)]
    if tensor_items:
        det = torch.zeros((), device=device)
        for v in tensor_items:
            c = torch.clamp(v, min=0.0, max=100.0)
            det = det + torch.where(torch.isfinite(c), c, torch.zeros_like(c))
        det = torch.clamp(det, min=0.0, max=500.0)
        adv = -1.0 * det
        if l2.requires_grad:
            adv = adv + (-10.0 * (l2 - 0.05))
        adv = torch.clamp(adv, min=-10.0, max=10.0)
        adv = torch.where((det > 0) & torch.isfinite(det), adv, torch.zeros_like(adv))
    else:
        adv = _zero(device)
    losses["loss_adversarial"] = adv
    if loss_dict is not None:
        zero = lambda: _zero(device)
        li = loss_dict.get("intensity_loss", None)
        lb = loss_dict.get("bias_loss", None)
        lm = loss_dict.get("imbalance_loss", None)
        losses["loss_intensity"] = 3.0 * li if (li is not None and li.requires_grad) else zero()
        losses["loss_bias"] = 10.0 * lb if (lb is not None and lb.requires_grad) else zero()
        losses["loss_imbalance"] = 10.0 * lm if (lm is not None and lm.requires_grad) else zero()
        losses["loss_adversarial"] = losses["loss_adversarial"] + 0.01 * (
            losses["loss_intensity"] + losses["loss_bias"] + losses["loss_imbalance"])
        reg_scale = max(0.1, 1.0 - ((epoch + 1) / 30.0))
        l2d = l2.detach()
        mult = torch.where(l2d < 0.001, 0.01, torch.where(l2d < 0.005, 0.1, torch.where(l2d < 0.01, 0.3, 1.0)))
        losses["loss_l2_regularization"] = (regularization_weight * reg_scale) * mult.to(l2.dtype) * l2
    else:
        for k in ("loss_intensity", "loss_bias", "loss_imbalance", "loss_l2_regularization"):
            losses[k] = _zero(device)
    losses["perturbation_l2_norm"] = l2.detach()
    return losses


def parse_losses(losses: dict):
    """mmengine BaseModel.parse_losses: total = sum of means of every key containing 'loss'
    (lists: sum of their means); returns (total, log_vars). A FusedLosses dict already holds the
    total (same sum, same order, computed in the loss-tail kernel)."""
    if isinstance(losses, FusedLosses):
        log_vars = {k: (v[0] if isinstance(v, list) else v) for k, v in losses.items()}
        return losses.total, dict(loss=losses.total, **log_vars)
    log_vars = {}
    for k, v in losses.items():
        if isinstance(v, torch.Tensor):
            log_vars[k] = v.mean()
        elif isinstance(v, (list, tuple)) and all(isinstance(t, torch.Tensor) for t in v):
            log_vars[k] = sum(t.mean() for t in v)
        else:
            raise TypeError(f"{k} is not a tensor or list of tensors")
    total = sum(v for k, v in log_vars.items() if "loss" in k)
    return total, dict(loss=total, **log_vars)
