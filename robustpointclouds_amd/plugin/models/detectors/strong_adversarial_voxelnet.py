"""StrongAdversarialVoxelNet — drop-in for models/detectors/strong_adversarial_voxelnet.py:13-324
(BASELINE config 5).

Same registry name, constructor, attributes (`_epoch`, `_iteration`, `_current_scaling`,
`_last_perturbations`, `_last_adversarial_loss`) and methods (`update_adversarial_strength`,
`apply_enhanced_perturbations`, `extract_feat`, `loss`, `predict`). The perturbation acts on the
HardSimpleVFE output (post-VFE, :207-215):

    scaled    = (adversary(x) - x) * scaling [+ momentum_alpha * last_scaled]     (:141-175)
    perturbed = x + scaled ; l2 = ||scaled||_2 -> attack history                  (:177-186)
    loss_adversarial = -w * scaling * det + 0.1 * momentum_alpha * last_adv       (:262-283)
    loss_l2_regularization = regularization_weight * l2                           (:286-288)
    anti-adaptation: with probability anti_adaptation_prob (torch.rand on the host RNG, :251-252)
    the detector losses are scaled by 0.1                                          (:297-301)

The combine, the norm, the dynamic scaling (epoch / attack-history boost / curriculum) and the
history itself run in one HIP kernel (csrc/strong.hip) with the history in a device ring: the
reference's per-step `l2.item()` (:180) and host-side history are replaced by device state, so the
step has no host synchronisation of its own. The adversary is the HIP VoxelPerturber.
"""
from __future__ import annotations

import ctypes as C
from typing import Optional

import torch

from robustpointclouds_amd import _ffi
from robustpointclouds_amd.registry import MODELS as _LOCAL_MODELS
from robustpointclouds_amd.voxelnet import VoxelNet

from .. import builder

try:  # register into mmdet3d too when it is installed
    from mmdet3d.registry import MODELS as _MM_MODELS
except Exception:  # pragma: no cover - mmdet3d absent in this image
    _MM_MODELS = None

RING = 64   # RPC_STRONG_RING


class StrongPerturbFn(torch.autograd.Function):
    """(x, adv_out) -> (perturbed, l2); also writes scaled, the device state and the ring."""

    @staticmethod
    def forward(ctx, x, adv_out, cfg, last, history, state, scaled):
        lib = _ffi.load()
        x = x.contiguous()
        adv_out = adv_out.contiguous()
        n = x.numel()
        perturbed = torch.empty_like(x)
        wsz = lib.rpc_strong_perturb_workspace_size()
        ws = _ffi.workspace(wsz, x.device)
        _ffi.check(lib.rpc_strong_perturb_forward(C.byref(cfg), _ffi.ptr(x), _ffi.ptr(adv_out),
                                                  _ffi.ptr(last) if last is not None else None, n,
                                                  _ffi.ptr(perturbed), _ffi.ptr(scaled), _ffi.ptr(history),
                                                  _ffi.ptr(state), _ffi.ptr(ws), wsz, _ffi.stream_of(x)),
                   "rpc_strong_perturb_forward")
        ctx.save_for_backward(scaled, state)
        ctx.n = n
        return perturbed, state[1].clone()

    @staticmethod
    def backward(ctx, gp, gl2):
        lib = _ffi.load()
        scaled, state = ctx.saved_tensors
        gx = torch.empty_like(scaled) if ctx.needs_input_grad[0] else None
        ga = torch.empty_like(scaled) if ctx.needs_input_grad[1] else None
        gp = gp.contiguous() if gp is not None else None
        gl2 = gl2.float().contiguous().view(1) if gl2 is not None else None
        _ffi.check(lib.rpc_strong_perturb_backward(_ffi.ptr(scaled), ctx.n, _ffi.ptr(state), _ffi.ptr(gp),
                                                   _ffi.ptr(gl2), _ffi.ptr(gx), _ffi.ptr(ga), _ffi.stream_of(scaled)),
                   "rpc_strong_perturb_backward")
        return gx, ga, None, None, None, None, None


def _register(cls):
    _LOCAL_MODELS.register_module(module=cls)
    if _MM_MODELS is not None:
        _MM_MODELS.register_module(module=cls, force=True)
    return cls


@_register
class StrongAdversarialVoxelNet(VoxelNet):
    def __init__(self, data_preprocessor=None, voxel_encoder=None, middle_encoder=None, backbone=None, neck=None,
                 bbox_head=None, train_cfg=None, test_cfg=None, adversary_cfg=None, adversarial_loss_weight=0.3,
                 regularization_weight=0.01, class_attack_weights=None, post_encoding_noise_scales=None,
                 dynamic_scaling=True, curriculum_learning=True, scaling_factor=1.5, max_scaling=5.0,
                 momentum_alpha=0.9, anti_adaptation_prob=0.1, **kwargs):
        super().__init__(voxel_encoder=voxel_encoder, middle_encoder=middle_encoder, backbone=backbone, neck=neck,
                         bbox_head=bbox_head, train_cfg=train_cfg, test_cfg=test_cfg,
                         data_preprocessor=data_preprocessor, init_cfg=kwargs.get("init_cfg"))
        self.adversary = builder.build_adversary(adversary_cfg) if adversary_cfg else None
        self.adversarial_loss_weight = adversarial_loss_weight
        self.regularization_weight = regularization_weight
        self.class_attack_weights = class_attack_weights or {"Car": 1.0, "Pedestrian": 2.0, "Cyclist": 1.5}
        self.post_encoding_noise_scales = post_encoding_noise_scales or {
            "Car": 0.2, "Pedestrian": 0.3, "Cyclist": 0.25, "default": 0.2}
        self.dynamic_scaling = dynamic_scaling
        self.curriculum_learning = curriculum_learning
        self.scaling_factor = scaling_factor           # stored, never read (as :92)
        self.max_scaling = max_scaling
        self.momentum_alpha = momentum_alpha
        self.anti_adaptation_prob = anti_adaptation_prob
        self._epoch = 0
        self._iteration = 0
        self._attack_count = 0                         # len of the reference's _attack_history (untrimmed)
        self._history: Optional[torch.Tensor] = None   # device ring of the last RING l2 values
        self._state: Optional[torch.Tensor] = None     # device [scaling, l2, dynamic weight]
        self._last_perturbations: Optional[torch.Tensor] = None
        self._last_adversarial_loss: Optional[torch.Tensor] = None

    # ------------------------------------------------------------------ dynamic scaling (:109-139)
    def _host_scaling(self):
        """(epoch_scaling, complexity) — the parts of update_adversarial_strength that depend only on
        host counters; the attack-history boost is applied on the device."""
        epoch_scaling = min(1.0 + (self._epoch * 0.1), self.max_scaling)
        complexity = min(1.0 + (self._iteration / 10000.0), 2.0)
        return epoch_scaling, complexity

    def update_adversarial_strength(self):
        """Returns the scaling of the last perturbation step as a device scalar (1.0 when dynamic
        scaling is off); the value for the next step is formed inside the perturbation kernel."""
        if not self.dynamic_scaling:
            return 1.0
        return self._state[0] if self._state is not None else 1.0

    @property
    def _current_scaling(self) -> float:
        return float(self._state[0]) if self._state is not None else 1.0

    @property
    def _attack_history(self):
        """The most recent l2 norms (up to RING) — host copy, for inspection only."""
        if self._history is None:
            return []
        n = min(self._attack_count, RING)
        idx = [(self._attack_count - n + k) % RING for k in range(n)]
        return self._history[idx].cpu().tolist()

    # ------------------------------------------------------------------ perturbation (:141-192)
    def apply_enhanced_perturbations(self, voxel_features, training=True):
        if not training or self.adversary is None:
            return voxel_features, 0.0
        dev = voxel_features.device
        if self._history is None or self._history.device != dev:
            self._history = torch.zeros(RING, dtype=torch.float32, device=dev)
            self._state = torch.zeros(3, dtype=torch.float32, device=dev)
        out = self.adversary(voxel_features)
        adv_out = out[0] if isinstance(out, tuple) else voxel_features + out
        last = self._last_perturbations
        if last is not None and tuple(last.shape) != tuple(voxel_features.shape):
            last = None                                # momentum reset on a shape change (:166-175)
        epoch_scaling, complexity = self._host_scaling()
        cfg = _ffi.RpcStrongCfg()
        cfg.epoch_scaling, cfg.complexity, cfg.max_scaling = epoch_scaling, complexity, float(self.max_scaling)
        cfg.adversarial_loss_weight = float(self.adversarial_loss_weight)
        cfg.momentum_alpha = float(self.momentum_alpha)
        cfg.dynamic, cfg.curriculum = int(self.dynamic_scaling), int(self.curriculum_learning)
        cfg.history_count = self._attack_count
        scaled = torch.empty_like(voxel_features, dtype=torch.float32)
        perturbed, l2 = StrongPerturbFn.apply(voxel_features.float(), adv_out.float(), cfg,
                                              last.contiguous() if last is not None else None, self._history,
                                              self._state, scaled)
        self._last_perturbations = scaled
        self._attack_count += 1
        return perturbed, l2

    # ------------------------------------------------------------------ detector (:194-239)
    def extract_feat(self, batch_inputs_dict, batch_data_samples=None):
        self._iteration += 1
        vd = batch_inputs_dict["voxels"]
        self._sync_engines(vd["voxels"].device)
        feats = self.voxel_encoder(vd["voxels"], vd["num_points"], vd["coors"])
        if self.training and self.adversary is not None:
            feats, l2 = self.apply_enhanced_perturbations(feats, True)
            batch_inputs_dict["adversarial_l2_norm"] = l2
        B = batch_inputs_dict.get("batch_size") or int(vd["coors"][:, 0].max().item()) + 1   # :218
        x = self.middle_encoder(feats, vd["coors"], B)
        x = self.backbone(x)
        if self.neck is not None:
            x = self.neck(x)
        return x

    def loss(self, batch_inputs_dict, batch_data_samples, **kwargs):
        skip_detector_update = self.training and torch.rand(1).item() < self.anti_adaptation_prob   # :251-252
        x = self.extract_feat(batch_inputs_dict, batch_data_samples)
        losses = dict(self.bbox_head.loss(x, batch_data_samples, **kwargs))
        if self.training and self.adversary is not None:
            dev = self._state.device
            detection_loss = torch.tensor(0.0, device=dev, requires_grad=True)
            for k, v in losses.items():
                if "loss" in k and isinstance(v, torch.Tensor):
                    detection_loss = detection_loss + v
            # dynamic weight = adversarial_loss_weight * scaling (Python-float product, rounded once:
            # state[2] of the perturbation kernel)
            adversarial_loss = (-self._state[2]) * detection_loss
            if self._last_adversarial_loss is not None:                                    # :274-277
                adversarial_loss = adversarial_loss + 0.1 * (self.momentum_alpha * self._last_adversarial_loss)
            self._last_adversarial_loss = adversarial_loss.detach()
            if "adversarial_l2_norm" in batch_inputs_dict:
                losses["loss_l2_regularization"] = self.regularization_weight * batch_inputs_dict["adversarial_l2_norm"]
            losses["loss_adversarial"] = adversarial_loss
            if skip_detector_update:                                                       # :297-301
                for key in list(losses.keys()):
                    if key not in ("loss_adversarial", "loss_l2_regularization") and isinstance(losses[key],
                                                                                               torch.Tensor):
                        losses[key] = losses[key] * 0.1
        return losses

    @torch.no_grad()
    def predict(self, batch_inputs_dict, batch_data_samples=None, **kwargs):
        x = self.extract_feat(batch_inputs_dict, batch_data_samples)
        return self.bbox_head(x)

