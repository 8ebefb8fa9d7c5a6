"""Dense BEV backbone + neck.

`SECOND` / `SECONDFPN` restate upstream mmdet3d backbones/second.py and necks/second_fpn.py
as configured at configs/adversarial/adversarial-second_hv_secfpn_8xb6-80e_kitti-3d-3class.py:25-36
(called at models/detectors/adversarial_voxelnet.py:142-145): Conv3x3-BN-ReLU stacks, BN eps
1e-3 momentum 0.01, conv bias off; FPN deconvs (kernel = stride) + BN + ReLU, concatenated.
These are the MFMA-bound layers. With `hip = True` (set by the Trainer) the whole stack runs as one
HIP node per module on the dense engine of dense_bev.py — bf16 MFMA in the perf mode (bench.py), fp32
MFMA (dense_f32.hip) in the parity mode; the plain torch path below is the reference / CPU form.
Module names match mmdet3d state dicts.
"""
from __future__ import annotations

import torch
from torch import nn


def _bn2d(c, norm_cfg):
    return nn.BatchNorm2d(c, eps=norm_cfg.get("eps", 1e-3), momentum=norm_cfg.get("momentum", 0.01))


class SECOND(nn.Module):
    def __init__(self, in_channels=128, out_channels=(128, 128, 256), layer_nums=(3, 5, 5),
                 layer_strides=(2, 2, 2), norm_cfg=dict(type="BN", eps=1e-3, momentum=0.01),
                 conv_cfg=dict(type="Conv2d", bias=False), init_cfg=None, pretrained=None):
        super().__init__()
        assert len(layer_strides) == len(layer_nums) == len(out_channels)
        in_filters = [in_channels, *out_channels[:-1]]
        blocks = []
        for i, n in enumerate(layer_nums):
            layers = [nn.Conv2d(in_filters[i], out_channels[i], 3, stride=layer_strides[i], padding=1, bias=False),
                      _bn2d(out_channels[i], norm_cfg), nn.ReLU(inplace=True)]
            for _ in range(n):
                layers += [nn.Conv2d(out_channels[i], out_channels[i], 3, padding=1, bias=False),
                           _bn2d(out_channels[i], norm_cfg), nn.ReLU(inplace=True)]
            blocks.append(nn.Sequential(*layers))
        self.blocks = nn.ModuleList(blocks)
        for m in self.modules():   # init_cfg = Kaiming on Conv2d (mmdet3d default)
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
        self.hip = False   # perf mode: the whole stack as one HIP implicit-GEMM node (dense_bev.py)

    def forward(self, x):
        if self.hip:
            from .dense_bev import second_forward
            return second_forward(self, x)
        outs = []
        for b in self.blocks:
            x = b(x)
            outs.append(x)
        return tuple(outs)


class SECONDFPN(nn.Module):
    def __init__(self, in_channels=(128, 128, 256), out_channels=(256, 256, 256), upsample_strides=(1, 2, 4),
                 norm_cfg=dict(type="BN", eps=1e-3, momentum=0.01), upsample_cfg=dict(type="deconv", bias=False),
                 conv_cfg=dict(type="Conv2d", bias=False), use_conv_for_no_stride=False, init_cfg=None):
        super().__init__()
        assert len(out_channels) == len(upsample_strides) == len(in_channels)
        deblocks = []
        for i, oc in enumerate(out_channels):
            s = upsample_strides[i]
            if s > 1 or (s == 1 and not use_conv_for_no_stride):
                up = nn.ConvTranspose2d(in_channels[i], oc, int(s), stride=int(s), bias=False)
            else:
                k = int(round(1 / s))
                up = nn.Conv2d(in_channels[i], oc, k, stride=k, bias=False)
            deblocks.append(nn.Sequential(up, _bn2d(oc, norm_cfg), nn.ReLU(inplace=True)))
        self.deblocks = nn.ModuleList(deblocks)
        for m in self.modules():
            if isinstance(m, nn.ConvTranspose2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
        self.hip = False   # perf mode: deblocks + concat as one HIP node (dense_bev.py)

    def forward(self, x):
        if self.hip:
            from .dense_bev import fpn_forward
            return fpn_forward(self, x)
        ups = [d(x[i]) for i, d in enumerate(self.deblocks)]
        return [torch.cat(ups, dim=1) if len(ups) > 1 else ups[0]]
