"""PARITY ORACLE — TEST INFRASTRUCTURE ONLY (tests/ and smoke() import it; the product never does).

CPU restatement of upstream mmdet3d `HardVFE` (mmdet3d/models/voxel_encoders/voxel_encoder.py,
class HardVFE + VFELayer; the "VFE per-voxel PointNet MLP+max" that BASELINE.json's north_star
names). mmdet3d is not vendored in /root/reference (`mmdetection3d/` is an empty
directory) and the reference ships no HardVFE vectors, so this restatement is **parity unpinned**
w.r.t. mmdet3d itself; it is checked against an independent pure-Python loop on small cases
(tests/test_oracle_hard_vfe.py). Semantics restated (mmdet3d 1.x):

* feature decoration, in this order: the raw F features, then (with_cluster_center) xyz minus the
  voxel's point mean — the sum runs over ALL max_points slots (padded slots are zero) divided by
  num_points —, then (with_voxel_center) xyz minus the voxel centre `coor * voxel_size +
  voxel_size / 2 + pc_range_min` (coors are (b, z, y, x)), then (with_distance) the L2 norm of xyz;
* the decorated [V, T, C0] tensor is multiplied by the padding mask (slot < num_points);
* every VFELayer: Linear(bias=False) -> BatchNorm1d over all V*T rows (padded rows included:
  BN1d runs on the permuted [V, C, T] tensor) -> ReLU -> max over the T slots; all but the last
  layer concatenate [pointwise, repeated max] (width 2C) as the next layer's input, the last returns
  the max [V, C];
* BatchNorm1d(eps=1e-3, momentum=0.01) by default (HardVFE's norm_cfg); train mode normalises with
  the biased batch variance and updates running_var with the unbiased one.

Everything runs in torch float64 (default) with autograd for the gradients.
"""
from __future__ import annotations

import torch


def decorate(features, num_points, coors, *, with_cluster_center, with_voxel_center, with_distance,
             voxel_size, point_cloud_range):
    """[V, T, F] -> masked decorated [V, T, C0] (HardVFE.forward, before the VFE layers)."""
    V, T, F = features.shape
    parts = [features]
    if with_cluster_center:
        mean = features[:, :, :3].sum(dim=1, keepdim=True) / num_points.to(features.dtype).view(-1, 1, 1)
        parts.append(features[:, :, :3] - mean)
    if with_voxel_center:
        c = coors.to(features.dtype)
        off = [voxel_size[i] / 2 + point_cloud_range[i] for i in range(3)]
        fc = torch.stack([features[:, :, 0] - (c[:, 3:4] * voxel_size[0] + off[0]),
                          features[:, :, 1] - (c[:, 2:3] * voxel_size[1] + off[1]),
                          features[:, :, 2] - (c[:, 1:2] * voxel_size[2] + off[2])], dim=-1)
        parts.append(fc)
    if with_distance:
        parts.append(torch.norm(features[:, :, :3], 2, 2, keepdim=True))
    x = torch.cat(parts, dim=-1)
    mask = (num_points.view(-1, 1) > torch.arange(T, device=features.device).view(1, -1))
    return x * mask.unsqueeze(-1).to(x.dtype)


def vfe_layer(x, W, gamma, beta, rm, rv, *, last, training, eps=1e-3, momentum=0.01, keep=None):
    """VFELayer.forward on [V, T, K] -> [V, T, 2C] (cat_max) or [V, C] (last). Updates rm / rv in
    place in training mode (as nn.BatchNorm1d). keep (a list) receives the pre-ReLU values."""
    V, T, _ = x.shape
    y = x @ W.T                                                    # [V, T, C]
    if training:
        flat = y.reshape(-1, y.shape[-1])
        mean = flat.mean(0)
        var = flat.var(0, unbiased=False)
        n = flat.shape[0]
        with torch.no_grad():
            rm.mul_(1 - momentum).add_(momentum * mean.detach())
            rv.mul_(1 - momentum).add_(momentum * (var.detach() * n / max(n - 1, 1)))
    else:
        mean, var = rm, rv
    z = (y - mean) / torch.sqrt(var + eps) * gamma + beta
    if keep is not None:
        keep.append(z.detach())
    p = torch.relu(z)
    m = p.max(dim=1, keepdim=True)[0]
    if last:
        return m.squeeze(1)
    return torch.cat([p, m.expand(V, T, m.shape[-1])], dim=2)


def hard_vfe(features, num_points, coors, layers, *, with_cluster_center=False, with_voxel_center=False,
             with_distance=False, voxel_size=(0.2, 0.2, 4), point_cloud_range=(0, -40, -3, 70.4, 40, 1),
             training=True, eps=1e-3, momentum=0.01, keep=None):
    """HardVFE.forward. `layers` = list of dicts with W [C, K], gamma, beta, rm, rv (tensors);
    keep (a list) receives every layer's pre-ReLU [V, T, C] values."""
    x = decorate(features, num_points, coors, with_cluster_center=with_cluster_center,
                 with_voxel_center=with_voxel_center, with_distance=with_distance, voxel_size=voxel_size,
                 point_cloud_range=point_cloud_range)
    for i, L in enumerate(layers):
        x = vfe_layer(x, L["W"], L["gamma"], L["beta"], L["rm"], L["rv"], last=(i == len(layers) - 1),
                      training=training, eps=eps, momentum=momentum, keep=keep)
    return x


def loop_hard_vfe(features, num_points, coors, layers, cfg):
    """Independent pure-Python-loop forward (float64 scalars) for small cases: decoration, Linear,
    batch statistics, BN, ReLU and the slot max written element by element."""
    import math
    V, T, F = features.shape
    f = features.tolist()
    npv = num_points.tolist()
    co = coors.tolist()
    vs, pr = cfg["voxel_size"], cfg["point_cloud_range"]
    X = []
    for v in range(V):
        mean = [sum(f[v][t][d] for t in range(T)) / npv[v] for d in range(3)]
        rows = []
        for t in range(T):
            r = list(f[v][t])
            if cfg.get("with_cluster_center"):
                r += [f[v][t][d] - mean[d] for d in range(3)]
            if cfg.get("with_voxel_center"):
                cen = [co[v][3] * vs[0] + vs[0] / 2 + pr[0], co[v][2] * vs[1] + vs[1] / 2 + pr[1],
                       co[v][1] * vs[2] + vs[2] / 2 + pr[2]]
                r += [f[v][t][d] - cen[d] for d in range(3)]
            if cfg.get("with_distance"):
                r += [math.sqrt(sum(f[v][t][d] ** 2 for d in range(3)))]
            rows.append([val if t < npv[v] else 0.0 for val in r])
        X.append(rows)
    eps = cfg.get("eps", 1e-3)
    for i, L in enumerate(layers):
        W = L["W"].tolist()
        g, b = L["gamma"].tolist(), L["beta"].tolist()
        C = len(W)
        Y = [[[sum(W[c][k] * X[v][t][k] for k in range(len(W[c]))) for c in range(C)] for t in range(T)]
             for v in range(V)]
        n = V * T
        mu = [sum(Y[v][t][c] for v in range(V) for t in range(T)) / n for c in range(C)]
        var = [sum((Y[v][t][c] - mu[c]) ** 2 for v in range(V) for t in range(T)) / n for c in range(C)]
        P = [[[max(0.0, (Y[v][t][c] - mu[c]) / math.sqrt(var[c] + eps) * g[c] + b[c]) for c in range(C)]
              for t in range(T)] for v in range(V)]
        M = [[max(P[v][t][c] for t in range(T)) for c in range(C)] for v in range(V)]
        if i == len(layers) - 1:
            return M
        X = [[P[v][t] + M[v] for t in range(T)] for v in range(V)]
    return X
