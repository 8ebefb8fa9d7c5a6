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

import contextlib
import math
import os
import warnings

import torch
import torch.distributed as dist

import robustpointclouds_amd.plugin.models  # noqa: F401  (registers AdversarialVoxelNet, VoxelPerturber)

from . import _ffi
from .base_model import ddp_train_step, select_engines
from .optim import ClipAdamW, OptimWrapper
from .registry import MODELS
from .voxelnet import second_kitti_cfg, second_kitti_strong_cfg


# Trainer._prefetch also builds the next batch's sparse rulebooks (RPC_PREFETCH_RULEBOOKS=0: off, A/B)
PREFETCH_RULEBOOKS = os.environ.get("RPC_PREFETCH_RULEBOOKS", "1") != "0"


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


def build_optim_wrapper(model, cfg: dict):
    """mmengine `build_optim_wrapper` for the reference configs' `optim_wrapper` dict
    (…3class.py:130-139): type OptimWrapper | AmpOptimWrapper (dtype 'bfloat16' / 'float16'),
    optimizer AdamW(lr, betas, eps, weight_decay), clip_grad(max_norm, norm_type 2), paramwise_cfg
    custom_keys lr_mult. On a ROCm device the optimizer is ClipAdamW (clip + AdamW, two launches).
    AmpOptimWrapper with dtype 'float16' or None (fp16 + GradScaler in mmengine) is run as bf16 autocast
    without a scaler, with a warning: the HIP engines have no fp16 path."""
    cfg = dict(cfg)
    kind = cfg.get("type", "OptimWrapper")
    oc = dict(cfg["optimizer"])
    if oc.pop("type", "AdamW") != "AdamW":
        raise ValueError("only AdamW (the reference configs' optimizer) is supported")
    lr = float(oc["lr"])
    betas = tuple(oc.get("betas", (0.9, 0.999)))
    eps, wd = float(oc.get("eps", 1e-8)), float(oc.get("weight_decay", 1e-2))
    keys = (cfg.get("paramwise_cfg") or {}).get("custom_keys", {})
    groups = param_groups(model, lr, keys)
    clip = cfg.get("clip_grad")
    dev = next(model.parameters()).device
    if dev.type == "cuda":
        opt = ClipAdamW(groups, lr=lr, betas=betas, eps=eps, weight_decay=wd,
                        max_norm=float(clip["max_norm"]) if clip else 0.0)
    else:
        opt = torch.optim.AdamW(groups, lr=lr, betas=betas, eps=eps, weight_decay=wd)
    amp = None
    if kind == "AmpOptimWrapper":
        dt = cfg.get("dtype")
        if dt not in ("bfloat16", "float16", None):
            raise ValueError(f"AmpOptimWrapper dtype {dt!r}: 'bfloat16', 'float16' or None")
        if dt != "bfloat16":
            # mmengine: None / 'float16' = fp16 autocast with a GradScaler (the reference's --amp,
            # trainUpdated.bat:9). The HIP engines have no fp16 path: bf16 autocast (fp32 exponent range,
            # so no loss scaler) is substituted
            warnings.warn(f"AmpOptimWrapper dtype {dt!r} (fp16 + GradScaler in mmengine) runs as bfloat16 "
                          "autocast without a loss scaler on the HIP engines", stacklevel=2)
        amp = torch.bfloat16
    elif kind != "OptimWrapper":
        raise ValueError(f"optim_wrapper type {kind}")
    return OptimWrapper(opt, clip_grad=clip, amp_dtype=amp)


class LRSchedule:
    """mmengine's chained param_scheduler of the reference configs (…3class.py:142-159):

        LinearLR(start_factor 0.1, by_epoch=False, begin 0, end 2000)
        CosineAnnealingLR(T_max 30, eta_min 1e-6, begin 0, end 30, by_epoch=True,
                          convert_to_iter_based=True)  -> T_max = end = 30 * iters_per_epoch

    restated RECURSIVELY, as mmengine applies them: each scheduler rescales the group's CURRENT lr
    once per iteration (ParamSchedulerHook.after_train_iter), so a manual lr change by a hook
    (NaNDetectionHook's x0.1) persists, and eta_min is the same absolute floor for every group
    (no eta_min_ratio). Construction applies step 0 (LinearLR: lr = initial_lr * start_factor)."""

    def __init__(self, optimizer, iters_per_epoch, warmup=2000, start_factor=0.1, T_max=30, eta_min=1e-6,
                 cos_end=None):
        self.opt = optimizer
        self.ipe = max(1, iters_per_epoch)
        self.start = start_factor
        self.lin_end = warmup                       # LinearLR end (iterations)
        self.lin_total = warmup - 1                 # mmengine: total_iters = end - begin - 1
        self.T = T_max * self.ipe                   # convert_to_iter_based
        self.cos_end = (T_max if cos_end is None else cos_end) * self.ipe
        self.eta_min = eta_min
        for g in optimizer.param_groups:
            g.setdefault("initial_lr", g["lr"])
        self.base = [g["initial_lr"] for g in optimizer.param_groups]
        self.last_step = 0
        if self.lin_end > 0:
            for g in optimizer.param_groups:
                g["lr"] = g["lr"] * self.start

    def step(self):
        """After one training iteration: LinearLR.step() then CosineAnnealingLR.step()."""
        self.last_step += 1
        t = self.last_step
        gs = self.opt.param_groups
        if t < self.lin_end and self.lin_total > 0:
            f = 1.0 + (1.0 - self.start) / (self.lin_total * self.start + (t - 1) * (1.0 - self.start))
            for g in gs:
                g["lr"] = g["lr"] * f
        if t < self.cos_end:
            T, eta = self.T, self.eta_min
            if (t - 1 - T) % (2 * T) == 0:
                for g, b in zip(gs, self.base):
                    g["lr"] = g["lr"] + (b - eta) * (1 - math.cos(math.pi / T)) / 2
            else:
                r = (1 + math.cos(math.pi * t / T)) / (1 + math.cos(math.pi * (t - 1) / T))
                for g in gs:
                    g["lr"] = r * (g["lr"] - eta) + eta

    def state_dict(self):
        return dict(last_step=self.last_step)

    def load_state_dict(self, sd):
        self.last_step = int(sd["last_step"])


class Trainer:
    def __init__(self, model, lr=1e-4, weight_decay=1e-3, betas=(0.9, 0.999), eps=1e-8, max_norm=0.5,
                 iters_per_epoch=1000, ddp=False, bf16=False, device=None):
        self.device = device or torch.device("cuda", torch.cuda.current_device())
        self.module = model.to(self.device)
        self.model = model
        if self.device.type == "cuda":
            self._select_engines(model, bf16)
        if ddp and dist.is_initialized():
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
        self._next = None        # (points, ready event) of the next batch, prefetched in update_params

    @staticmethod
    def _select_engines(model, bf16):
        # pinned: evaluation (val_step outside autocast) keeps the training precision's engines
        select_engines(model, bf16, pin=True)

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

    def train_step(self, points, gt, next_points=None, next_ready=None):
        """points: list of [Ni, 4] cuda tensors; gt: dict(gt_boxes [B, M, 7], gt_labels [B, M]).

        next_points (optional): the next step's points. Their hard voxelisation and sparse rulebooks
        are queued on side streams during this step — after its backward has been issued, so the host
        reads they need (the voxel count, the strided convolutions' output counts) block the host while
        the GPU still has this step's work queued — and the next step's forward starts with both ready.
        next_ready (optional): an event after which next_points are complete (default: everything queued
        on the training stream before this step). Same kernels, same results: only where and when the
        voxelisation and the rulebooks are queued changes."""
        m = self.module
        if not m.training:
            m.train()
        pend = self._pending
        self._pending = None
        if pend is not None and pend[0] is points:
            v, c, n, vn = pend[1].result(torch.cuda.current_stream(self.device))
            batch = dict(points=points, voxels=dict(voxels=v, coors=c, num_points=n, voxel_num=vn))
        else:   # voxelised by the model's data_preprocessor inside train_step, as mmengine does
            batch = dict(points=points)
        batch["batch_size"] = len(points)
        self._next = None
        if next_points is not None and self.device.type == "cuda":
            if next_ready is None:
                next_ready = torch.cuda.Event()
                next_ready.record(torch.cuda.current_stream(self.device))
            self._next = (next_points, next_ready)
        out = self.step_batch(batch, gt)
        self._issue_prefetch()      # no-op when update_params already issued it
        return out

    def _issue_prefetch(self):
        nxt = getattr(self, "_next", None)
        self._next = None
        if nxt is not None:
            self._prefetch(*nxt)

    def _prefetch(self, points, after):
        vl = getattr(getattr(self.module, "data_preprocessor", None), "voxel_layer", None)
        if vl is None or not hasattr(vl, "voxelize_frames_deferred") or self.device.type != "cuda":
            return
        if self._side is None:
            self._side = _ffi.side_stream(self.device)
        vl.train(True)
        for p in points:    # read on the side stream: keep the allocator from reusing them early
            p.record_stream(self._side)
        # the points may still be in flight on the training stream (GpuTrainAugment output, a
        # non_blocking pinned copy): order the side stream after the caller's readiness event
        self._side.wait_event(after)
        with torch.cuda.stream(self._side):
            pend = vl.voxelize_frames_deferred(points)
        self._pending = (points, pend)
        # and that batch's sparse rulebooks: their host reads (V, four strided output counts) happen now,
        # while the GPU still runs this step's queued work, so next step's sparse forward issues its
        # GEMMs without waiting on the GPU
        me = getattr(self.module, "middle_encoder", None)
        if PREFETCH_RULEBOOKS and me is not None and hasattr(me, "prepare"):
            V = pend.count()
            me.prepare(pend.t[1][:V], len(points), after=pend.ev, consumer=torch.cuda.current_stream(self.device))

    def step_batch(self, batch, gt):
        """The step after voxelisation, as mmengine runs it: model.train_step(data, optim_wrapper)
        (MMDistributedDataParallel.train_step under DDP) with this trainer as the optim wrapper —
        loss -> parse_losses -> backward (DDP all-reduce) -> clip -> AdamW — then the hooks and the
        LR schedule. batch: dict(voxels=dict(voxels, num_points, coors), batch_size); gt: the
        padded dict(gt_boxes, gt_labels) or mmdet3d Det3DDataSamples."""
        m = self.module
        if not m.training:   # Module.train() walks every submodule (~1 ms of host time)
            m.train()
        data = dict(inputs=batch, data_samples=gt)
        if isinstance(self.model, torch.nn.parallel.DistributedDataParallel):
            log_vars = ddp_train_step(self.model, data, self)    # DDP hooks fire on the grads
        else:
            log_vars = m.train_step(data, self)
        self.iter += 1
        self.last_log = log_vars
        # hooks first, then the schedulers (mmengine: NaNDetectionHook NORMAL priority runs before
        # ParamSchedulerHook LOW), so a hook's lr cut is what the schedule rescales from
        for h in self.hooks:
            if hasattr(h, "after_train_iter"):
                h.after_train_iter(self, self.iter - 1, None, log_vars)
        self.sched.step()
        return log_vars

    # ------------------------------------------------------------------ mmengine OptimWrapper surface
    def optim_context(self, model):
        """AmpOptimWrapper.optim_context: autocast (bf16) in the perf mode, nothing in fp32."""
        return torch.autocast("cuda", dtype=torch.bfloat16) if self.bf16 else contextlib.nullcontext()

    def update_params(self, loss):
        """OptimWrapper.update_params: backward, clip_grad (max_norm 0.5) + AdamW, zero_grad. The batch
        prefetch (train_step next_points) is issued here, right after the backward: its host reads
        then block while the GPU still has the whole backward queued."""
        loss.backward()
        self._issue_prefetch()
        if isinstance(self.opt, ClipAdamW):
            self._grad_norm = self.opt.step()[0]
        else:
            self._grad_norm = torch.nn.utils.clip_grad_norm_(self.module.parameters(), self.max_norm)
            self.opt.step()
        self.opt.zero_grad(set_to_none=True)


def make_kitti_model(num_classes=1, device=None, adversarial=True, hidden_channels=None, epoch=3, variant="voxelnet"):
    """variant 'voxelnet': AdversarialVoxelNet (configs/adversarial/...kitti-3d-{car,3class}.py);
    'strong': StrongAdversarialVoxelNet with sensor_error_bound 0.4 (BASELINE config 5)."""
    if variant == "strong":
        cfg = second_kitti_strong_cfg(num_classes, hidden_channels=hidden_channels)
    else:
        cfg = second_kitti_cfg(num_classes, hidden_channels=hidden_channels, adversarial=adversarial)
    model = build_model(cfg)
    model._epoch = epoch
    if device is not None:
        model.to(device)
    return model


def make_nus_model(device=None, adversarial=True, epoch=3):
    """AdversarialCenterPoint on the nuScenes CenterPoint stack (configs/adversarial/
    adversarial-centerpoint_voxel-nuscenes.py, BASELINE config 4)."""
    from .centerpoint import centerpoint_nus_cfg
    model = build_model(centerpoint_nus_cfg(adversarial=adversarial))
    model._epoch = epoch
    if device is not None:
        model.to(device)
    return model


def init_distributed(force: bool = False):
    """torch.distributed from torchrun env vars; backend nccl (= RCCL on ROCm) on GPU, gloo on CPU.

    A process launched by torch.distributed.run (RANK in the environment) always joins a process
    group, also at WORLD_SIZE 1, so a one-rank run still builds the RCCL communicator and sends
    DDP's bucketed all-reduce through it; a plain `python` run (no RANK) stays single-process
    unless `force` (then a one-rank group on 127.0.0.1)."""
    if "RANK" not in os.environ:
        if not force:
            return 0, 1, 0
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(_free_port()))
        os.environ.update(RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    rank = int(os.environ["RANK"])
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", rank))
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    # nccl (= RCCL) on GPU; RPC_DIST_BACKEND=gloo lets several ranks share one GPU in tests
    backend = os.environ.get("RPC_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
    if torch.cuda.is_available():
        torch.cuda.set_device(local % torch.cuda.device_count())
    if not dist.is_initialized():
        dist.init_process_group(backend=backend)
    return rank, world, local


def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]
