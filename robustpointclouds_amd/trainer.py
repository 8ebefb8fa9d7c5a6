"""One adversarial training step, end to end (SURVEY.md §3.1, §8(a) rows a1–a11).

    Det3DDataPreprocessor.voxelize (HIP) -> AdversarialVoxelNet.loss -> parse_losses
    -> backward (HIP kernels + MIOpen, DDP bucketed all-reduce over RCCL)
    -> clip_grad_norm(0.5) -> AdamW (adversary lr_mult 2.0) -> LR schedule

restating the mmengine Runner / OptimWrapper flow that train.py:120-128 drives with
configs/adversarial/adversarial-second_hv_secfpn_8xb6-80e_kitti-3d-3class.py:130-159.
Data-parallel: one process per GPU, frames sharded across ranks; perturber std / BN
statistics stay per rank (no SyncBN, like the reference).
"""
from __future__ import annotations

import math
import os

import torch
import torch.distributed as dist

import robustpointclouds_amd.plugin.models  # noqa: F401  (registers AdversarialVoxelNet, VoxelPerturber)

from .adversarial_loss import parse_losses
from .optim import ClipAdamW
from .registry import MODELS
from .voxelnet import second_kitti_cfg, second_kitti_strong_cfg


def build_model(cfg: dict):
    return MODELS.build(cfg)


def param_groups(model, lr, custom_keys=None):
    """mmengine DefaultOptimWrapperConstructor paramwise_cfg custom_keys={'adversary': lr_mult 2.0}."""
    custom_keys = custom_keys if custom_keys is not None else {"adversary": dict(lr_mult=2.0)}
    groups = {}
    for name, p in model.named_parameters():
        if not p.requires_grad:
            continue
        mult = 1.0
        for k, v in custom_keys.items():
            if k in name:
                mult = v.get("lr_mult", 1.0)
                break
        groups.setdefault(mult, []).append(p)
    return [dict(params=ps, lr=lr * m, initial_lr=lr * m) for m, ps in sorted(groups.items())]


class LRSchedule:
    """LinearLR(start 0.1, 2000 iters) then CosineAnnealingLR(T_max epochs, eta_min) (:142-159)."""

    def __init__(self, optimizer, iters_per_epoch, warmup=2000, start_factor=0.1, T_max=30, eta_min=1e-6):
        self.opt = optimizer
        self.ipe = max(1, iters_per_epoch)
        self.warmup, self.start, self.T, self.eta_min = warmup, start_factor, T_max, eta_min
        self.base = [g["initial_lr"] for g in optimizer.param_groups]

    def set(self, it):
        w = 1.0 if it >= self.warmup else self.start + (1.0 - self.start) * it / self.warmup
        ep = min(it / self.ipe, self.T)
        for g, b in zip(self.opt.param_groups, self.base):
            eta = self.eta_min * b / self.base[0]
            cos = eta + (b - eta) * (1 + math.cos(math.pi * ep / self.T)) / 2
            g["lr"] = cos * w


class Trainer:
    def __init__(self, model, lr=1e-4, weight_decay=1e-3, betas=(0.9, 0.999), eps=1e-8, max_norm=0.5,
                 iters_per_epoch=1000, ddp=False, bf16=False, device=None):
        self.device = device or torch.device("cuda", torch.cuda.current_device())
        self.module = model.to(self.device)
        self.model = model
        if bf16 and getattr(model, "middle_encoder", None) is not None and hasattr(model.middle_encoder, "bf16"):
            # perf mode: sparse convs on bf16 MFMA; dense BEV handed over as a bf16 NHWC image to
            # SECOND / SECONDFPN on the HIP dense-conv engine and the HIP head (the images are
            # channels_last; the parameters keep torch's contiguous layout, so gradients are stolen
            # by AccumulateGrad without layout copies)
            model.middle_encoder.bf16 = True
            model.middle_encoder.dense_nhwc = True
            model.middle_encoder.dense_bf16 = True
            for name in ("backbone", "neck", "pts_backbone", "pts_neck"):
                mod = getattr(model, name, None)
                if mod is None:
                    continue
                if hasattr(mod, "hip"):
                    mod.hip = True
                else:
                    mod.to(memory_format=torch.channels_last)
        if ddp and dist.is_initialized() and dist.get_world_size() > 1:
            # 6 MB buckets: the 16 MB of SECOND gradients (ready together when its one-node backward
            # ends) go out in three RCCL all-reduces that overlap the sparse-encoder and perturber
            # backward; with one 25 MB bucket the reduction waited for the end of backward
            self.model = torch.nn.parallel.DistributedDataParallel(
                model, device_ids=[self.device.index] if self.device.type == "cuda" else None,
                bucket_cap_mb=6, find_unused_parameters=False, broadcast_buffers=False, gradient_as_bucket_view=True)
        if self.device.type == "cuda":
            # clip_grad_norm_ + AdamW as two HIP kernels over a device tensor table (optim.py)
            self.opt = ClipAdamW(param_groups(self.module, lr), lr=lr, betas=betas, eps=eps,
                                 weight_decay=weight_decay, max_norm=max_norm)
        else:   # host-only runs (the gloo DDP test of the distributed logic): torch's optimizer
            self.opt = torch.optim.AdamW(param_groups(self.module, lr), lr=lr, betas=betas, eps=eps,
                                         weight_decay=weight_decay)
        self.sched = LRSchedule(self.opt, iters_per_epoch)
        self.max_norm = max_norm
        self.bf16 = bf16
        self.iter = 0
        self.epoch = 0
        self.hooks = []
        self.should_stop = False
        self.last_log = None
        self._side = None        # side stream of the batch prefetch
        self._pending = None     # (points list, PendingVoxels) of the prefetched next batch

    # mmengine-runner-like attributes used by custom_hook.py
    @property
    def optim_wrapper(self):
        return self

    @property
    def optimizer(self):
        return self.opt

    def register_hook(self, hook):
        self.hooks.append(hook)

    def before_epoch(self):
        for h in self.hooks:
            if hasattr(h, "before_train_epoch"):
                h.before_train_epoch(self)

    def train_step(self, points, gt, next_points=None):
        """points: list of [Ni, 4] cuda tensors; gt: dict(gt_boxes [B, M, 7], gt_labels [B, M]).

        next_points (optional): the next step's points, already complete on the device. Their hard
        voxelisation is queued on a side stream now, concurrently with this step, and its voxel count
        is read at the next step, so that read no longer drains the training stream (the next step's
        kernels queue behind this step's backward instead of starting on an idle GPU). Same kernels,
        same results: only where the voxelisation is queued changes."""
        m = self.module
        if not m.training:
            m.train()
        pend = self._pending
        self._pending = None
        if pend is not None and pend[0] is points:
            v, c, n, vn = pend[1].result(torch.cuda.current_stream(self.device))
            batch = dict(points=points, voxels=dict(voxels=v, coors=c, num_points=n, voxel_num=vn))
        else:
            batch = m.data_preprocessor(dict(inputs=dict(points=points)), training=True)["inputs"]
        batch["batch_size"] = len(points)
        if next_points is not None:
            self._prefetch(next_points)
        return self.step_batch(batch, gt)

    def _prefetch(self, points):
        vl = getattr(getattr(self.module, "data_preprocessor", None), "voxel_layer", None)
        if vl is None or not hasattr(vl, "voxelize_frames_deferred") or self.device.type != "cuda":
            return
        if self._side is None:
            self._side = torch.cuda.Stream(self.device)
        vl.train(True)
        for p in points:    # read on the side stream: keep the allocator from reusing them early
            p.record_stream(self._side)
        with torch.cuda.stream(self._side):
            self._pending = (points, vl.voxelize_frames_deferred(points))

    def step_batch(self, batch, gt):
        """The step after voxelisation: loss -> parse_losses -> backward (DDP all-reduce) -> clip
        -> AdamW -> hooks. batch: dict(voxels=dict(voxels, num_points, coors), batch_size)."""
        m = self.module
        if not m.training:   # Module.train() walks every submodule (~1 ms of host time)
            m.train()
        self.sched.set(self.iter)
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=self.bf16):
            if isinstance(self.model, torch.nn.parallel.DistributedDataParallel):
                losses = self.model(batch, gt, mode="loss")     # DDP hooks fire on the grads
            else:
                losses = m.loss(batch, gt)
        total, log_vars = parse_losses(losses)
        total.backward()
        if isinstance(self.opt, ClipAdamW):
            self._grad_norm = self.opt.step()[0]
        else:
            self._grad_norm = torch.nn.utils.clip_grad_norm_(self.module.parameters(), self.max_norm)
            self.opt.step()
        self.opt.zero_grad(set_to_none=True)
        self.iter += 1
        self.last_log = log_vars
        for h in self.hooks:
            if hasattr(h, "after_train_iter"):
                h.after_train_iter(self, self.iter - 1, None, log_vars)
        return log_vars


def _ddp_forward(self, batch, gt, mode="loss"):
    return self.loss(batch, gt)


def make_kitti_model(num_classes=1, device=None, adversarial=True, hidden_channels=None, epoch=3, variant="voxelnet"):
    """variant 'voxelnet': AdversarialVoxelNet (configs/adversarial/...kitti-3d-{car,3class}.py);
    'strong': StrongAdversarialVoxelNet with sensor_error_bound 0.4 (BASELINE config 5)."""
    if variant == "strong":
        cfg = second_kitti_strong_cfg(num_classes, hidden_channels=hidden_channels)
    else:
        cfg = second_kitti_cfg(num_classes, hidden_channels=hidden_channels, adversarial=adversarial)
    model = build_model(cfg)
    # DDP calls forward(); route it to loss() like mmengine's BaseModel.forward(mode='loss')
    model.forward = _ddp_forward.__get__(model)
    model._epoch = epoch
    if device is not None:
        model.to(device)
    return model


def make_nus_model(device=None, adversarial=True, epoch=3):
    """AdversarialCenterPoint on the nuScenes CenterPoint stack (configs/adversarial/
    adversarial-centerpoint_voxel-nuscenes.py, BASELINE config 4)."""
    from .centerpoint import centerpoint_nus_cfg
    model = build_model(centerpoint_nus_cfg(adversarial=adversarial))
    model.forward = _ddp_forward.__get__(model)
    model._epoch = epoch
    if device is not None:
        model.to(device)
    return model


def init_distributed():
    """torch.distributed from torchrun env vars; backend nccl (= RCCL on ROCm) on GPU, gloo on CPU."""
    if "RANK" not in os.environ or int(os.environ.get("WORLD_SIZE", "1")) <= 1:
        return 0, 1, 0
    rank = int(os.environ["RANK"])
    world = int(os.environ["WORLD_SIZE"])
    local = int(os.environ.get("LOCAL_RANK", rank))
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    # nccl (= RCCL) on GPU; RPC_DIST_BACKEND=gloo lets several ranks share one GPU in tests
    backend = os.environ.get("RPC_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
    if torch.cuda.is_available():
        torch.cuda.set_device(local % torch.cuda.device_count())
    if not dist.is_initialized():
        dist.init_process_group(backend=backend)
    return rank, world, local
