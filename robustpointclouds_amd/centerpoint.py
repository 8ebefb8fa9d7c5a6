"""CenterPoint (points branch) detector stack on this framework's kernels.

Restates upstream mmdet3d `CenterPoint` (detectors/centerpoint.py, an MVXTwoStageDetector whose
point modules carry the `pts_` prefix) as configured by the base of
configs/adversarial/adversarial-centerpoint_voxel-nuscenes.py:11-13
(centerpoint_voxel01_second_secfpn_head-dcn-circlenms_8xb4-cyclic-20e_nus-3d, not vendored):
hard voxelisation (0.1 x 0.1 x 0.2 m, 10 points, 90000 voxels) -> HardSimpleVFE(5) -> basicblock
SparseEncoder [41, 1024, 1024] -> SECOND [128, 256] -> SECONDFPN (conv for the stride-1 deblock) ->
CenterHead (six tasks, DCNSeparateHead). `AdversarialCenterPoint` (plugin/models/detectors)
subclasses it.
"""
from __future__ import annotations

import torch
from torch import nn

from .center_head import NUS_COMMON_HEADS, NUS_TASKS, NUS_TRAIN_CFG, CenterHead
from .base_model import DetectorBase
from .registry import MODELS
from .voxelnet import Det3DDataPreprocessor

MODELS.register_module(module=CenterHead)

NUS_PC_RANGE = [-51.2, -51.2, -5.0, 51.2, 51.2, 3.0]
NUS_VOXEL_SIZE = [0.1, 0.1, 0.2]


class CenterPoint(DetectorBase):
    def __init__(self, pts_voxel_encoder=None, pts_middle_encoder=None, pts_backbone=None, pts_neck=None,
                 pts_bbox_head=None, train_cfg=None, test_cfg=None, data_preprocessor=None, init_cfg=None, **kwargs):
        super().__init__()
        build = lambda c: c if (c is None or isinstance(c, nn.Module)) else MODELS.build(c)
        self.data_preprocessor = build(data_preprocessor) if data_preprocessor is not None else \
            Det3DDataPreprocessor()
        self.pts_voxel_encoder = build(pts_voxel_encoder)
        self.pts_middle_encoder = build(pts_middle_encoder)
        self.pts_backbone = build(pts_backbone)
        self.pts_neck = build(pts_neck)
        if pts_bbox_head is not None and not isinstance(pts_bbox_head, nn.Module):
            pts_bbox_head = dict(pts_bbox_head)
            pts_bbox_head.update(train_cfg=(train_cfg or {}).get("pts"), test_cfg=(test_cfg or {}).get("pts"))
        self.pts_bbox_head = build(pts_bbox_head)
        self.train_cfg = train_cfg
        self.test_cfg = test_cfg

    @property
    def with_pts_neck(self):
        return self.pts_neck is not None

    # aliases the trainer's perf-mode switches look for
    @property
    def middle_encoder(self):
        return self.pts_middle_encoder

    def _batch_size(self, voxel_dict):
        bs = voxel_dict.get("batch_size") if isinstance(voxel_dict, dict) else None
        return bs if bs else int(voxel_dict["coors"][-1, 0].item()) + 1    # upstream: coors[-1, 0] + 1

    def extract_pts_feat(self, voxel_dict, points=None, img_feats=None, batch_input_metas=None):
        self._sync_engines(voxel_dict["voxels"].device)
        feats = self.pts_voxel_encoder(voxel_dict["voxels"], voxel_dict["num_points"], voxel_dict["coors"])
        x = self.pts_middle_encoder(feats, voxel_dict["coors"], self._batch_size(voxel_dict))
        x = self.pts_backbone(x)
        if self.with_pts_neck:
            x = self.pts_neck(x)
        return x

    def _forward(self, inputs, data_samples=None, **kwargs):
        vd = dict(inputs["voxels"])
        vd.setdefault("batch_size", inputs.get("batch_size"))
        return self.pts_bbox_head(self.extract_pts_feat(vd))

    def loss(self, batch_inputs_dict, batch_data_samples, **kwargs):
        vd = dict(batch_inputs_dict["voxels"])
        vd.setdefault("batch_size", batch_inputs_dict.get("batch_size"))
        return self.pts_bbox_head.loss(self.extract_pts_feat(vd), batch_data_samples)


MODELS.register_module(module=CenterPoint)


def centerpoint_nus_cfg(adversarial=True, hidden_channels=(16, 32, 64)):
    """The model dict of configs/adversarial/adversarial-centerpoint_voxel-nuscenes.py resolved against
    its upstream centerpoint_voxel01_second_secfpn_head-dcn base (not vendored in /root/reference)."""
    norm = dict(type="BN", eps=1e-3, momentum=0.01)
    cfg = dict(
        type="AdversarialCenterPoint" if adversarial else "CenterPoint",
        data_preprocessor=dict(type="Det3DDataPreprocessor", voxel=True, voxel_type="hard",
                               voxel_layer=dict(max_num_points=10, voxel_size=NUS_VOXEL_SIZE,
                                                max_voxels=(90000, 120000), point_cloud_range=NUS_PC_RANGE)),
        pts_voxel_encoder=dict(type="HardSimpleVFE", num_features=5),
        pts_middle_encoder=dict(type="SparseEncoder", in_channels=5, sparse_shape=[41, 1024, 1024],
                                output_channels=128, order=("conv", "norm", "act"),
                                encoder_channels=((16, 16, 32), (32, 32, 64), (64, 64, 128), (128, 128)),
                                encoder_paddings=((0, 0, 1), (0, 0, 1), (0, 0, [0, 1, 1]), (1, 1)),
                                block_type="basicblock"),
        pts_backbone=dict(type="SECOND", in_channels=256, out_channels=[128, 256], layer_nums=[5, 5],
                          layer_strides=[1, 2], norm_cfg=norm, conv_cfg=dict(type="Conv2d", bias=False)),
        pts_neck=dict(type="SECONDFPN", in_channels=[128, 256], out_channels=[256, 256], upsample_strides=[1, 2],
                      norm_cfg=norm, upsample_cfg=dict(type="deconv", bias=False), use_conv_for_no_stride=True),
        pts_bbox_head=dict(type="CenterHead", in_channels=512,
                           tasks=[dict(num_class=len(t), class_names=list(t)) for t in NUS_TASKS],
                           common_heads=dict(NUS_COMMON_HEADS), share_conv_channel=64, norm_bbox=True,
                           loss_cls_weight=1.0, loss_bbox_weight=0.25, init_bias=-2.19),
        train_cfg=dict(pts=dict(NUS_TRAIN_CFG)),
        test_cfg=dict(pts=dict(post_center_limit_range=[-61.2, -61.2, -10.0, 61.2, 61.2, 10.0], max_per_img=500,
                               max_pool_nms=False, min_radius=[4, 12, 10, 1, 0.85, 0.175], score_threshold=0.1,
                               out_size_factor=8, voxel_size=NUS_VOXEL_SIZE[:2], nms_type="circle",
                               pre_max_size=1000, post_max_size=83, nms_thr=0.2)))
    if adversarial:
        cfg.update(adversary_cfg=dict(type="VoxelPerturber", sensor_error_bound=0.2, voxel_size=NUS_VOXEL_SIZE,
                                      use_spatial_attention=True, hidden_channels=list(hidden_channels)),
                   adversarial_loss_weight=0.05, regularization_weight=0.005)
    return cfg
