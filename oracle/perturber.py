"""PARITY ORACLE — TEST INFRASTRUCTURE ONLY (tests/, smoke(), bench cpu_baseline).

CPU restatement of the VoxelPerturber forward/backward
(/root/reference/models/adversarial/voxel_perturber.py) and of the valid-slot compaction +
masked scatter + HardSimpleVFE of AdversarialVoxelNet.extract_feat
(/root/reference/models/detectors/adversarial_voxelnet.py:85-137), written with explicit
torch ops on CPU (float64 by default, for an accurate reference; float32 to mimic the
reference bit-for-bit as far as op order allows).

Pinned against golden vectors produced by running the reference itself
(tests/golden/make_golden.py -> tests/golden/perturber_*.npz), see
tests/test_oracle_golden.py.
"""
from __future__ import annotations

import numpy as np
import torch


def bounds(F: int, training: bool, e: float = 0.2, dtype=torch.float32):
    """(scale, clamp) vectors with the float32 op order of voxel_perturber.py:209-256, :333-359."""
    f32 = torch.float32
    eb = torch.ones(F, dtype=f32) * e
    if F == 4:
        if not training:                                    # :214-231
            eb = eb * (2.5 * ((2.0 + 1.5 + 1.2) / 3.0))
            eb[:3] *= 2.0
            eb[3] = 1.5
            cb = torch.ones(F, dtype=f32) * e * 5.0         # :341-344
            cb[:3] *= 5.0
            cb[3] = 2.0
        else:                                               # :241-244
            eb = eb * 0.8
            eb[:3] *= 1.3
            eb[3] = 0.2
            cb = torch.ones(F, dtype=f32) * e * 0.9         # :347-350
            cb[:3] *= 1.2
            cb[3] = 0.1
    else:                                                   # :251-253, :351-354
        eb[4:] = 0.0
        cb = torch.ones(F, dtype=f32) * e
        cb[4:] = 0.0
    return eb.to(dtype), cb.to(dtype)


class OraclePerturber:
    """Weights in the fixture naming: W0..W5, b0..b5 (Linear [out, in]), g0..g4 / be0..be4
    (BatchNorm affine), rm/rv running stats, Wa0/ba0/Wa1/ba1 (attention)."""

    def __init__(self, weights: dict, F: int, hidden, dtype=torch.float64, eps=1e-3, momentum=0.1,
                 use_attention=True, sensor_error_bound=0.2):
        self.F = F
        self.hidden = list(hidden)
        self.dtype = dtype
        self.eps = eps
        self.mom = momentum
        self.att = use_attention
        self.e = sensor_error_bound
        self.p = {}
        names = [f"W{l}" for l in range(6)] + [f"b{l}" for l in range(6)] + \
            [f"g{l}" for l in range(5)] + [f"be{l}" for l in range(5)] + \
            (["Wa0", "ba0", "Wa1", "ba1"] if use_attention else [])
        for k in names:
            t = torch.tensor(np.asarray(weights[k]), dtype=dtype)
            self.p[k] = t.requires_grad_(True)
        widths = [F] + [hidden[0], hidden[1], hidden[2], hidden[1], hidden[0]]
        self.rm = [torch.zeros(widths[l + 1], dtype=dtype) for l in range(5)]
        self.rv = [torch.ones(widths[l + 1], dtype=dtype) for l in range(5)]

    def forward(self, x, training=True):
        """x [N, F] -> (out, dict). Mirrors voxel_perturber.py:120-321."""
        p = self.p
        x = torch.as_tensor(x).to(self.dtype)
        s = torch.std(x, dim=0, keepdim=True) + 1e-6                       # :158
        if torch.isnan(s).any() or torch.isinf(s).any():                   # :161-163
            s = torch.ones_like(s)
        xn = torch.clamp(x / s, -10.0, 10.0)                               # :165-168
        h = xn
        for l in range(5):                                                 # :82-100
            z = h @ p[f"W{l}"].T + p[f"b{l}"]
            if training:
                mean = z.mean(0)
                var = z.var(0, unbiased=False)
                n = z.shape[0]
                with torch.no_grad():
                    self.rm[l] = (1 - self.mom) * self.rm[l] + self.mom * mean.detach()
                    self.rv[l] = (1 - self.mom) * self.rv[l] + self.mom * var.detach() * n / max(n - 1, 1)
            else:
                mean, var = self.rm[l], self.rv[l]
            z = (z - mean) / torch.sqrt(var + self.eps) * p[f"g{l}"] + p[f"be{l}"]
            h = torch.relu(z)
        raw = torch.tanh(h @ p["W5"].T + p["b5"])                          # :101-102
        if self.att:                                                       # :203-205
            a = torch.relu(xn @ p["Wa0"].T + p["ba0"])
            raw = raw * torch.sigmoid(a @ p["Wa1"].T + p["ba1"])
        eb, cb = bounds(self.F, training, self.e, self.dtype)
        pert = raw * eb.view(1, -1)                                        # :256
        pert = torch.clamp(pert, -cb.view(1, -1), cb.view(1, -1))         # :357-359
        pert = torch.nan_to_num(pert, nan=0.0)                             # :362-365
        l2 = torch.norm(pert, p=2, dim=1).mean()                           # :269
        out = x + pert                                                     # :285
        inten = pert[:, 3].abs().mean()                                    # :290
        bias = pert.mean(dim=0).abs().mean()                               # :295
        imb = pert.std(dim=0).std()                                        # :298-299
        return out, dict(l2_norm=l2, intensity_loss=inten, bias_loss=bias, imbalance_loss=imb)

    def grads(self):
        """Parameter grads after the reference's hook clamp(nan_to_num(g), -0.1, 0.1) (:465-475)."""
        out = {}
        for k, t in self.p.items():
            g = torch.zeros_like(t) if t.grad is None else t.grad
            out["d" + k] = torch.clamp(torch.nan_to_num(g, nan=0.0, posinf=0.0, neginf=0.0), -0.1, 0.1)
        return out

    def zero_grad(self):
        for t in self.p.values():
            t.grad = None


def perturb_voxels(op: OraclePerturber, voxels, num_points, vfe_features=4, training=True):
    """adversarial_voxelnet.py:85-117 + HardSimpleVFE: returns (vfe, perturbed voxels, dict)."""
    voxels = torch.as_tensor(voxels).to(op.dtype)
    V, P, F = voxels.shape
    flat = voxels.reshape(-1, F)
    valid = flat.sum(dim=1) != 0                                           # :89
    pv = flat[valid]
    out, ld = op.forward(pv, training)
    pert_flat = flat + torch.zeros_like(flat)                              # :113
    pert_flat = pert_flat.masked_scatter(valid[:, None].expand_as(flat), out)
    pert = pert_flat.view(V, P, F)
    npts = torch.as_tensor(num_points).to(op.dtype).view(-1, 1)
    vfe = pert[:, :, :vfe_features].sum(dim=1) / npts                      # HardSimpleVFE
    return vfe, pert, ld
