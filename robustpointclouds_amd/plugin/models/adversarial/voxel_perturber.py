"""VoxelPerturber — drop-in for models/adversarial/voxel_perturber.py:19-541.

Same registry name, constructor, nn.Sequential layout / state-dict keys
(`model.{0,3,6,9,12,15}` Linear, `model.{1,4,7,10,13}` BatchNorm1d, `attention.{0,2}`),
initialisation (:434-462) and `forward(x[N, F]) -> (x + pert, loss_dict)` semantics; the
arithmetic runs in the HIP kernels of robustpointclouds_amd.perturb (no CPU path).

Declared deviations (SURVEY.md findings 2, §5):
* the network is built EAGERLY in __init__ (the reference builds it on the first forward,
  :142-147, so its parameters miss the optimizer and DDP); F is guessed exactly as the
  reference does (:61) and the model is rebuilt lazily if a forward brings another F;
* the grad hook clamp(nan_to_num(g), -0.1, 0.1) (:465-475) is applied inside the backward
  kernel to each parameter's full gradient (identical values; no per-tensor hook launches);
* any hidden_channels up to 256 (the reference builds any widths, :82-103): widths the kernels
  are not instantiated for (8, 16, 32, 64, 128, 256) run zero-padded to the next one — padded Linear
  rows / columns and BatchNorm affine entries are zero, so a padded channel is identically 0 after
  its BatchNorm + ReLU and feeds nothing; the real channels' values, batch statistics and
  gradients are unchanged (autograd slices the padded gradients back), and the running
  statistics of the real channels are copied back after each forward;
* NaN input / NaN perturbations (:150-153, :195-200, :259-262) are detected on the device:
  the output is the unperturbed input and the loss terms are zeros (no host sync), and
  the per-step metrics (:388-409) are accumulated on the device and read only in
  save_l2_norms().
"""
from __future__ import annotations

import csv
import warnings
from typing import Tuple

import torch
from torch import nn

from robustpointclouds_amd import _ffi
from robustpointclouds_amd import perturb as _P

from ..builder import ADVERSARIES

_HIST_CAP = 1 << 16
_NATIVE = (8, 16, 32, 64, 128, 256)   # hidden widths the perturber kernels are instantiated for


def _native_width(c: int) -> int:
    for n in _NATIVE:
        if c <= n:
            return n
    raise ValueError(f"VoxelPerturber: hidden width {c} > {_NATIVE[-1]} is not supported by the HIP kernels")


class _GradHookClamp(torch.autograd.Function):
    """Identity on a parameter whose backward is the reference's per-parameter grad hook
    clamp(nan_to_num(g, 0, 0, 0), -0.1, 0.1) (voxel_perturber.py:465-475). Each perturber
    parameter is used once per forward, so clamping its one incoming gradient here is the hook."""

    @staticmethod
    def forward(ctx, p):
        return p.view_as(p)

    @staticmethod
    def backward(ctx, g):
        return torch.clamp(torch.nan_to_num(g, nan=0.0, posinf=0.0, neginf=0.0), -0.1, 0.1)


def _bounds_torch(F: int, training: bool, e: float, device):
    """(forward scale, clamp) vectors of voxel_perturber.py:209-256 / :333-359 in the same fp32 op
    order (KITTI F = 4 train / eval; F > 4: bound e, timestamp channels 0)."""
    eb = torch.ones(F, device=device) * e
    if F == 4:
        if not training:
            eb *= 2.5 * ((2.0 + 1.5 + 1.2) / 3.0)
            eb[:3] *= 2.0
            eb[3] = 1.5
            cb = torch.ones(F, device=device) * e * 5.0
            cb[:3] *= 5.0
            cb[3] = 2.0
        else:
            eb *= 0.8
            eb[:3] *= 1.3
            eb[3] = 0.2
            cb = torch.ones(F, device=device) * e * 0.9
            cb[:3] *= 1.2
            cb[3] = 0.1
    elif F > 4:
        eb[4:] = 0.0
        cb = torch.ones(F, device=device) * e
        cb[4:] = 0.0
    else:
        raise ValueError(f"VoxelPerturber: {F} input features (the reference defines bounds for F >= 4)")
    return eb, cb


class PackedLosses(dict):
    """The reference's loss dict; `.packed` is the device vector its entries are views of."""
    packed = None


@ADVERSARIES.register_module(force=True)
class VoxelPerturber(nn.Module):
    def __init__(self, sensor_error_bound: float = 0.2, voxel_size: list = [0.05, 0.05, 0.1],
                 use_spatial_attention: bool = True, hidden_channels: list = [8, 16, 32]):
        super().__init__()
        self.sensor_error_bound = float(sensor_error_bound)
        self.voxel_size = torch.tensor(list(voxel_size))
        self.use_spatial_attention = use_spatial_attention
        self.voxel_error_bound = sensor_error_bound / torch.tensor(list(voxel_size) + [1.0])
        self.auto_detect_dims = True
        in_features = 5 if (voxel_size[0] >= 0.1 or voxel_size[2] >= 0.15) else 4
        self.in_features = in_features
        if len(hidden_channels) < 3:
            raise ValueError(f"hidden_channels needs 3 entries (encoder-decoder widths), got {hidden_channels}")
        # the reference reads hidden_channels[0..2] only (:82-103) and ignores extra entries
        # (configs/adversarial/adversarial-second_strong_v2.py passes [64, 128, 256, 128])
        self.hidden_channels = [int(c) for c in list(hidden_channels)[:3]]
        self._kernel_hidden = [_native_width(int(c)) for c in self.hidden_channels]
        self._bound_max = float(self.voxel_error_bound.max())
        self.model = None
        self.attention = None
        self.l2_norms = []
        self.l2_percentages = []
        self.constraint_violations = []
        self.perturbation_stats = []
        self._hist = None
        self._hist_n = 0
        self._build_model(in_features)

    # ------------------------------------------------------------------ build / init
    def _build_model(self, num_features):
        h = self.hidden_channels
        dev = self.model[0].weight.device if self.model is not None else None
        self.model = nn.Sequential(
            nn.Linear(num_features, h[0]), nn.BatchNorm1d(h[0]), nn.ReLU(inplace=True),
            nn.Linear(h[0], h[1]), nn.BatchNorm1d(h[1]), nn.ReLU(inplace=True),
            nn.Linear(h[1], h[2]), nn.BatchNorm1d(h[2]), nn.ReLU(inplace=True),
            nn.Linear(h[2], h[1]), nn.BatchNorm1d(h[1]), nn.ReLU(inplace=True),
            nn.Linear(h[1], h[0]), nn.BatchNorm1d(h[0]), nn.ReLU(inplace=True),
            nn.Linear(h[0], num_features), nn.Tanh())
        if self.use_spatial_attention:
            a = max(num_features // 2, 1)
            self.attention = nn.Sequential(nn.Linear(num_features, a), nn.ReLU(inplace=True), nn.Linear(a, 1),
                                           nn.Sigmoid())
        self.in_features = num_features
        self._init_weights()
        if dev is not None:
            self.to(dev)

    def _init_weights(self):
        for m in self.modules():                                  # :439-462
            if isinstance(m, nn.Linear):
                if m.out_features in (4, 5):
                    std = 0.025 if m.out_features == 4 else 0.01
                    nn.init.normal_(m.weight, 0.0, std)
                    if m.bias is not None:
                        nn.init.normal_(m.bias, 0.0, std)
                else:
                    nn.init.xavier_uniform_(m.weight, gain=1.0)
                    if m.bias is not None:
                        nn.init.constant_(m.bias, 0)
            elif isinstance(m, nn.BatchNorm1d):
                nn.init.constant_(m.weight, 1)
                nn.init.constant_(m.bias, 0)
                m.momentum = 0.1
                m.eps = 1e-3

    def _reset_problematic_weights(self):
        """:477-497 (only called on NaN detection, so its host reads are off the hot path)."""
        with torch.no_grad():
            for m in self.modules():
                if isinstance(m, nn.Linear):
                    if torch.isnan(m.weight).any():
                        nn.init.xavier_uniform_(m.weight, gain=0.001)
                    if m.bias is not None and torch.isnan(m.bias).any():
                        nn.init.constant_(m.bias, 0)
                elif isinstance(m, nn.BatchNorm1d):
                    if torch.isnan(m.weight).any():
                        nn.init.constant_(m.weight, 1)
                    if torch.isnan(m.bias).any():
                        nn.init.constant_(m.bias, 0)
                    if torch.isnan(m.running_mean).any():
                        nn.init.constant_(m.running_mean, 0)
                    if torch.isnan(m.running_var).any():
                        nn.init.constant_(m.running_var, 1)

    # ------------------------------------------------------------------ kernel plumbing
    def _padded(self):
        return self._kernel_hidden != self.hidden_channels

    def kernel_params(self):
        """36 tensors in rpc_perturber order (include/rpc_hip.h); zero-padded to the kernel widths
        when hidden_channels are not native (differentiable pads: gradients slice back)."""
        lin = [m for m in self.model if isinstance(m, nn.Linear)]
        bns = [m for m in self.model if isinstance(m, nn.BatchNorm1d)]
        ps = []
        if not self._padded():
            for l in range(5):
                ps += [lin[l].weight, lin[l].bias, bns[l].weight, bns[l].bias, bns[l].running_mean,
                       bns[l].running_var]
            ps += [lin[5].weight, lin[5].bias]
        else:
            F = self.in_features
            h = self._kernel_hidden
            kw = [F, h[0], h[1], h[2], h[1], h[0], F]
            pad = nn.functional.pad
            rs = self._running_pads(bns, kw)
            for l in range(6):
                W, b = lin[l].weight, lin[l].bias
                po, pi = kw[l + 1] - W.shape[0], kw[l] - W.shape[1]
                ps += [pad(W, (0, pi, 0, po)), pad(b, (0, po))]
                if l < 5:
                    bn = bns[l]
                    ps += [pad(bn.weight, (0, po)), pad(bn.bias, (0, po)), rs[l][0], rs[l][1]]
        if self.use_spatial_attention:
            att = [m for m in self.attention if isinstance(m, nn.Linear)]
            ps += [att[0].weight, att[0].bias, att[1].weight, att[1].bias]
        else:
            ps += [None] * 4
        return ps

    def _running_pads(self, bns, kw):
        """Padded running-stat buffers (the kernel updates them in place), refreshed from the
        modules' own buffers; _sync_running copies the real channels back after the forward."""
        dev = bns[0].running_mean.device
        if getattr(self, "_rpad", None) is None or self._rpad[0][0].device != dev:
            self._rpad = [(torch.zeros(kw[l + 1], device=dev), torch.ones(kw[l + 1], device=dev)) for l in range(5)]
        with torch.no_grad():
            for (rm, rv), bn in zip(self._rpad, bns):
                c = bn.running_mean.shape[0]
                rm[:c].copy_(bn.running_mean)
                rv[:c].copy_(bn.running_var)
        return self._rpad

    def _sync_running(self):
        if not self._padded() or not self.training:
            return
        bns = [m for m in self.model if isinstance(m, nn.BatchNorm1d)]
        with torch.no_grad():
            for (rm, rv), bn in zip(self._rpad, bns):
                c = bn.running_mean.shape[0]
                bn.running_mean.copy_(rm[:c])
                bn.running_var.copy_(rv[:c])

    def _cfg(self, F, vfe_features=4):
        bn = [m for m in self.model if isinstance(m, nn.BatchNorm1d)][0]
        return _P.make_cfg(F, self._kernel_hidden, self.use_spatial_attention, self.training,
                           self.sensor_error_bound, bn.eps, bn.momentum, vfe_features,
                           getattr(self, "wgrad_split_bf16", False), getattr(self, "act16", 0))

    def _ensure_width(self, F):
        if F != self.in_features:
            warnings.warn(f"VoxelPerturber: rebuilding for {F} input features (built for {self.in_features}); "
                          "the new parameters are not in an optimizer created before this call")
            self._build_model(F)

    def _bump_batch_counts(self):
        if self.training:
            _ffi.bump_batches([m for m in self.model if isinstance(m, nn.BatchNorm1d)])

    @staticmethod
    def _loss_dict(lvec):
        d = PackedLosses(l2_norm=lvec[0], intensity_loss=lvec[1], bias_loss=lvec[2], imbalance_loss=lvec[3])
        d.packed = lvec   # the [4] device vector the entries view (the fused loss tail reads it)
        return d

    # ------------------------------------------------------------------ forward
    def forward(self, voxel_features: torch.Tensor) -> Tuple[torch.Tensor, dict]:
        """ROCm tensors run the fused HIP kernels (and fail loudly if librpc_hip.so is missing);
        CPU tensors run the module's own torch layers (BASELINE configs[0], the reference's own
        device-agnostic torch path) — a dispatch on the input's device, never a fallback."""
        assert voxel_features.dim() == 2, f"Expected 2D input, got {voxel_features.dim()}D"
        self._ensure_width(voxel_features.shape[1])
        if voxel_features.device.type == "cpu":
            return self._forward_torch(voxel_features)
        x = voxel_features.float()
        out, lvec, flags = _P.PerturberFn.apply(x, self._cfg(x.shape[1]), *self.kernel_params())
        self._sync_running()
        self._bump_batch_counts()
        if self.training:
            self._track(lvec, out.detach() - x.detach(), x.detach().norm(dim=1).mean())
        return out, self._loss_dict(lvec)

    # ------------------------------------------------------------------ host (CPU) path
    def _forward_torch(self, x: torch.Tensor) -> Tuple[torch.Tensor, dict]:
        """voxel_perturber.py:120-321 + _apply_physical_constraints (:323-386) in torch on the host,
        op for op: unbiased std-normalisation (:158-168), the encoder-decoder MLP with train-mode
        BatchNorm (batch statistics, running-stat update, :176), the sigmoid attention gate
        (:203-205), bound scaling (:209-256), clamp + nan_to_num (:357-365) and the four loss terms
        (:268-299). The grad hook (:465-475) is an identity node on each parameter. NaN input / NaN
        perturbations return the unperturbed input and zero losses (the HIP path's device-flag
        behaviour)."""
        dev = x.device
        zeros = lambda: {k: torch.zeros((), device=dev) for k in
                         ("l2_norm", "intensity_loss", "bias_loss", "imbalance_loss")}
        if torch.isnan(x).any():                                                    # :150-153
            return x, zeros()
        s = torch.std(x, dim=0, keepdim=True) + 1e-6                                # :158
        if torch.isnan(s).any() or torch.isinf(s).any():                            # :161-163
            s = torch.ones_like(s)
        xn = torch.clamp(x.clone() / s, -10.0, 10.0)                                # :157, 165-168
        h = xn
        hook = _GradHookClamp.apply
        mods = list(self.model)
        for m in mods:
            if isinstance(m, nn.Linear):
                h = nn.functional.linear(h, hook(m.weight), hook(m.bias))
            elif isinstance(m, nn.BatchNorm1d):
                if self.training:
                    m.num_batches_tracked.add_(1)
                h = nn.functional.batch_norm(h, m.running_mean, m.running_var, hook(m.weight), hook(m.bias),
                                             self.training, m.momentum, m.eps)
            elif isinstance(m, nn.ReLU):
                h = torch.relu(h)
            elif isinstance(m, nn.Tanh):
                h = torch.tanh(h)
            else:
                h = m(h)
        raw = h
        if torch.isnan(raw).any():                                                  # :195-200
            self._reset_problematic_weights()
            return x, zeros()
        if self.use_spatial_attention:                                              # :203-205
            a0, _, a1, _ = list(self.attention)
            att = nn.functional.linear(torch.relu(nn.functional.linear(xn, hook(a0.weight), hook(a0.bias))),
                                       hook(a1.weight), hook(a1.bias))
            raw = raw * torch.sigmoid(att)
        F = x.shape[1]
        eb, cb = _bounds_torch(F, self.training, self.sensor_error_bound, dev)
        pert = raw * eb.view(1, -1)                                                 # :256
        if torch.isnan(pert).any():                                                 # :259-262
            return x, zeros()
        pert = torch.clamp(pert, -cb.view(1, -1), cb.view(1, -1))                   # :357-359
        if torch.isnan(pert).any():                                                 # :362-365
            pert = torch.nan_to_num(pert, nan=0.0)
        ref_norm = torch.norm(x, p=2, dim=1).mean()                                 # :268
        l2 = torch.norm(pert, p=2, dim=1).mean()                                    # :269
        if self.training:                                                           # :281-282
            self._track(l2.detach().reshape(1), pert.detach(), ref_norm.detach())
        out = x + pert                                                              # :285
        inten = pert[:, 3].abs().mean()                                             # :290
        bias = pert.mean(dim=0).abs().mean()                                        # :295
        imb = pert.std(dim=0).std()                                                 # :298-299
        return out, dict(l2_norm=l2, intensity_loss=inten, bias_loss=bias, imbalance_loss=imb)

    def _perturb_voxels_torch(self, voxels, num_points, vfe_features):
        """adversarial_voxelnet.py:85-117 + HardSimpleVFE on the host: valid = slot sum != 0 (:89),
        perturb the compacted points, gradient-connected masked scatter (:113-117), slot mean."""
        V, P, F = voxels.shape
        flat = voxels.reshape(-1, F).float()
        valid = flat.sum(dim=1) != 0
        out, ld = self._forward_torch(flat[valid]) if bool(valid.any()) else (flat[valid], None)
        if ld is None:
            ld = {k: torch.zeros(()) for k in ("l2_norm", "intensity_loss", "bias_loss", "imbalance_loss")}
        pert = (flat + torch.zeros_like(flat)).masked_scatter(valid[:, None].expand_as(flat), out).view(V, P, F)
        vfe = pert[:, :, :vfe_features].sum(dim=1) / num_points.to(pert.dtype).view(-1, 1)
        flags = torch.zeros(8)
        flags[4] = valid.sum()
        return vfe, ld, pert.detach(), flags

    def perturb_voxels(self, voxels: torch.Tensor, num_points: torch.Tensor, vfe_features: int = 4):
        """Fused path of AdversarialVoxelNet.extract_feat (adversarial_voxelnet.py:85-137):
        valid-slot mask + perturber + masked scatter + HardSimpleVFE in one kernel sequence.
        Returns (vfe [V, vfe_features], loss_dict, perturbed voxels, flags)."""
        self._ensure_width(voxels.shape[-1])
        if voxels.device.type == "cpu":
            return self._perturb_voxels_torch(voxels, num_points, vfe_features)
        vfe, lvec, pert, flags = _P.PerturbVoxelsFn.apply(voxels.float(), num_points,
                                                          self._cfg(voxels.shape[-1], vfe_features),
                                                          *self.kernel_params())
        self._sync_running()
        self._bump_batch_counts()
        if self.training:
            self._track(lvec, None, None)
        return vfe, self._loss_dict(lvec), pert, flags

    # ------------------------------------------------------------------ metrics
    def _track(self, lvec, pert, ref_norm):
        """Device-side version of _track_metrics (:388-409): no .item() per step."""
        if self._hist is None or self._hist.device != lvec.device:
            self._hist = torch.zeros((_HIST_CAP, 6), dtype=torch.float32, device=lvec.device)
            self._hist_n = 0
        if self._hist_n >= _HIST_CAP:
            self._flush_hist()
        nan = torch.full((), float("nan"), device=lvec.device)
        l2 = lvec[0].detach()
        if pert is not None:
            mx = pert.abs().max()
            row = torch.stack([l2, l2 / (ref_norm + 1e-8) * 100,
                               torch.clamp(mx - self._bound_max, min=0.0), mx,
                               pert.abs().mean(), pert.std()])
        else:
            row = torch.stack([l2, nan, nan, nan, nan, nan])
        self._hist[self._hist_n] = row
        self._hist_n += 1

    def _flush_hist(self):
        if self._hist is None or self._hist_n == 0:
            return
        h = self._hist[: self._hist_n].cpu().tolist()
        for l2, pct, viol, mx, mean, std in h:
            self.l2_norms.append(l2)
            self.l2_percentages.append(pct)
            self.constraint_violations.append(viol)
            self.perturbation_stats.append(dict(l2_norm=l2, l2_percentage=pct, max_perturbation=mx,
                                                mean_perturbation=mean, std_perturbation=std,
                                                constraint_violation=viol))
        self._hist_n = 0

    def save_l2_norms(self, filename="l2_norms.csv"):
        """:411-432 — CSV of the tracked metrics, then clear them."""
        self._flush_hist()
        with open(filename, "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["L2 Norm", "L2 Percentage", "Constraint Violations"])
            for n, p, v in zip(self.l2_norms, self.l2_percentages,
                               self.constraint_violations or [0] * len(self.l2_norms)):
                w.writerow([n, p, v])
        if self.perturbation_stats:
            with open(filename.replace(".csv", "_detailed.csv"), "w", newline="") as f:
                w = csv.DictWriter(f, fieldnames=self.perturbation_stats[0].keys())
                w.writeheader()
                w.writerows(self.perturbation_stats)
        self.l2_norms.clear()
        self.l2_percentages.clear()
        self.constraint_violations.clear()
        self.perturbation_stats.clear()
