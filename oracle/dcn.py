"""PARITY ORACLE — TEST INFRASTRUCTURE ONLY (tests/).

CPU restatement of mmcv `DeformConv2d` (deform_conv2d, stride 1, padding 1, dilation 1, kernel 3,
groups G, deform_groups 1) as used by the DCNSeparateHead of the CenterPoint base named at
configs/adversarial/adversarial-centerpoint_voxel-nuscenes.py:11-13. mmcv (requirements.txt:9) is
not vendored and no reference test holds vectors for it: parity is UNPINNED w.r.t. mmcv; this
restates its published CUDA semantics (deformable_im2col_bilinear: sample point outside
(-1, H) x (-1, W) -> 0, corners outside the image -> 0; offset channel 2k = dy, 2k + 1 = dx of tap
k = 3i + j). Gradients (input, offsets, weights) by torch autograd of the bilinear expression,
which equal mmcv's col2im / col2im_coord analytic gradients (floor() carries none).
"""
from __future__ import annotations

import torch


def deform_conv2d(x, offset, weight, groups=4):
    """x [B, C, H, W], offset [B, 18, H, W], weight [Co, C/groups, 3, 3] -> [B, Co, H, W]."""
    B, C, H, W = x.shape
    Co = weight.shape[0]
    cg, og = C // groups, Co // groups
    ys = torch.arange(H, dtype=x.dtype).view(1, H, 1)
    xs = torch.arange(W, dtype=x.dtype).view(1, 1, W)
    out = x.new_zeros((B, Co, H, W))
    flat = x.reshape(B, C, H * W)
    for k in range(9):
        i, j = k // 3, k % 3
        ph = ys - 1 + i + offset[:, 2 * k]
        pw = xs - 1 + j + offset[:, 2 * k + 1]
        valid = (ph > -1) & (pw > -1) & (ph < H) & (pw < W)
        hl = torch.floor(ph).detach()
        wl = torch.floor(pw).detach()
        lh, lw = ph - hl, pw - wl
        hh, hw = 1 - lh, 1 - lw
        val = x.new_zeros((B, C, H, W))
        for dy, dx, wgt in ((0, 0, hh * hw), (0, 1, hh * lw), (1, 0, lh * hw), (1, 1, lh * lw)):
            cy, cx = hl + dy, wl + dx
            ok = (cy >= 0) & (cy <= H - 1) & (cx >= 0) & (cx <= W - 1)
            idx = (cy.clamp(0, H - 1) * W + cx.clamp(0, W - 1)).long().view(B, 1, H * W).expand(B, C, H * W)
            v = flat.gather(2, idx).view(B, C, H, W)
            val = val + (wgt * ok).unsqueeze(1) * v
        col = val * valid.unsqueeze(1)
        for g in range(groups):
            wk = weight[g * og:(g + 1) * og, :, i, j]                           # [og, cg]
            out[:, g * og:(g + 1) * og] = out[:, g * og:(g + 1) * og] + torch.einsum(
                "oc,bchw->bohw", wk, col[:, g * cg:(g + 1) * cg])
    return out
