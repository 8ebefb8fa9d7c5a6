"""PARITY ORACLE — TEST INFRASTRUCTURE ONLY (tests/).

CPU restatement of StrongAdversarialVoxelNet's per-step logic (§8(f4)):
models/detectors/strong_adversarial_voxelnet.py
  update_adversarial_strength   :109-139  epoch scaling, attack-history boost, curriculum
  apply_enhanced_perturbations  :141-192  (adversary(x) - x) * scaling + momentum, l2, history
  extract_feat                  :194-239  VFE first, perturb the VFE output, middle / backbone / neck
  loss                          :241-303  anti-adaptation draw, -w*scaling*det + 0.1*alpha*last_adv,
                                          l2 regularisation, 0.1x detector losses when skipping
with the adversary a CPU OraclePerturber. Pinned against golden vectors from the reference itself
(tests/golden/strong_*.npz, tests/golden/make_golden.py:gen_strong).
"""
from __future__ import annotations

import numpy as np
import torch


class OracleStrong:
    def __init__(self, adversary, adversarial_loss_weight=0.3, regularization_weight=0.01, dynamic_scaling=True,
                 curriculum_learning=True, max_scaling=5.0, momentum_alpha=0.9, anti_adaptation_prob=0.1):
        self.adversary = adversary
        self.w, self.reg_w = adversarial_loss_weight, regularization_weight
        self.dynamic, self.curriculum = dynamic_scaling, curriculum_learning
        self.max_scaling, self.alpha, self.p_skip = max_scaling, momentum_alpha, anti_adaptation_prob
        self.epoch, self.iteration = 0, 0
        self.history = []
        self.scaling = 1.0
        self.last_pert = None
        self.last_adv = None

    def update_strength(self):
        if not self.dynamic:
            return 1.0
        s = min(1.0 + self.epoch * 0.1, self.max_scaling)
        if len(self.history) > 50:
            avg = np.mean([abs(v) for v in self.history[-50:]])
            s *= 2.0 if avg < 0.1 else (1.5 if avg < 0.3 else 1.0)
        if self.curriculum:
            s *= min(1.0 + self.iteration / 10000.0, 2.0)
        self.scaling = min(s, self.max_scaling)
        return self.scaling

    def perturb(self, x):
        s = self.update_strength()
        out, _ = self.adversary(x)
        scaled = (out - x) * s
        if self.last_pert is not None and self.last_pert.shape == scaled.shape:
            scaled = scaled + self.alpha * self.last_pert
        self.last_pert = scaled.detach()
        l2 = torch.norm(scaled, p=2)
        self.history.append(l2.item())
        if len(self.history) > 1000:
            self.history = self.history[-500:]
        return x + scaled, l2

    def loss(self, feats, coors, batch_size, middle, backbone, head, samples):
        """feats: the VFE output. Returns (losses dict, l2)."""
        skip = torch.rand(1).item() < self.p_skip
        self.iteration += 1
        feats, l2 = self.perturb(feats)
        x = backbone(middle(feats, coors, batch_size))
        losses = dict(head.loss(x, samples))
        det = torch.tensor(0.0, requires_grad=True)
        for k, v in losses.items():
            if "loss" in k and isinstance(v, torch.Tensor):
                det = det + v
        adv = -(self.w * self.scaling) * det
        if self.last_adv is not None:
            adv = adv + 0.1 * (self.alpha * self.last_adv)
        self.last_adv = adv.detach()
        losses["loss_l2_regularization"] = self.reg_w * l2
        losses["loss_adversarial"] = adv
        if skip:
            for k in list(losses):
                if k not in ("loss_adversarial", "loss_l2_regularization") and isinstance(losses[k], torch.Tensor):
                    losses[k] = losses[k] * 0.1
        return losses, l2
