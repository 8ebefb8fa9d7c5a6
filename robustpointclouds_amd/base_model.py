"""The mmengine `BaseModel` / mmdet3d `Base3DDetector` entry points the reference's Runner calls.

train.py:120-128 runs `Runner.from_cfg(cfg).train()`; each iteration mmengine calls
`model.train_step(data, optim_wrapper)` (through `MMDistributedDataParallel.train_step` under
`--launcher pytorch`), which runs

    with optim_wrapper.optim_context(model):
        data = model.data_preprocessor(data, True)          # Det3DDataPreprocessor: hard voxelize
        losses = model(**data, mode='loss')                 # AdversarialVoxelNet.loss (:153)
    parsed, log_vars = model.parse_losses(losses)
    optim_wrapper.update_params(parsed)                     # backward, clip, AdamW, zero_grad

and `val_step` / `test_step` run `mode='predict'`. `DetectorBase` restates that surface for this
build's detectors (VoxelNet / AdversarialVoxelNet / StrongAdversarialVoxelNet, CenterPoint /
AdversarialCenterPoint), so the plugin drops into the reference's runners unchanged; the build's
own `Trainer` drives the same `train_step`.

Engines: when a detector's tensors are on a ROCm device, its SparseEncoder / SECOND / SECONDFPN
run on the HIP engines (dense_bev.py, sparse_encoder.py). The precision follows torch autocast
like any torch op — inside `torch.autocast('cuda')` (mmengine's AmpOptimWrapper, `--amp`) the
bf16 MFMA perf mode, otherwise the fp32 parity mode — selected at the first forward and whenever
the autocast state changes (`select_engines`).
"""
from __future__ import annotations

from typing import Optional

import os

import torch
from torch import nn

from .adversarial_loss import parse_losses


def select_engines(model: nn.Module, bf16: bool, pin: bool = False) -> None:
    """Route the dense part through the HIP engines: bf16 perf mode (sparse convs on bf16 MFMA,
    dense BEV handed over as a bf16 NHWC image to SECOND / SECONDFPN on the bf16 dense engine and
    the bf16 head GEMM) or fp32 parity mode (fp32 sparse convs, an fp32 NHWC image through the
    fp32-MFMA dense engine and head GEMM). The images are channels_last; the parameters keep
    torch's contiguous layout (gradients are stolen by AccumulateGrad without layout copies)."""
    me = getattr(model, "middle_encoder", None) or getattr(model, "pts_middle_encoder", None)
    if me is not None and hasattr(me, "bf16"):
        me.bf16 = bool(bf16)
        me.dense_nhwc = True
        me.dense_bf16 = bool(bf16)
    for name in ("backbone", "neck", "pts_backbone", "pts_neck"):
        mod = getattr(model, name, None)
        if mod is None:
            continue
        if hasattr(mod, "hip"):
            mod.hip = True
        elif bf16:
            mod.to(memory_format=torch.channels_last)
    adv = getattr(model, "adversary", None)
    if adv is not None and hasattr(adv, "sensor_error_bound"):
        # perf mode: the perturber's hidden-layer weight gradients on split-bf16 MFMA (perturb.make_cfg);
        # RPC_PERT_SPLIT=0 keeps them on fp32 MFMA
        adv.wgrad_split_bf16 = bool(bf16) and os.environ.get("RPC_PERT_SPLIT", "1") != "0"
        # perf mode option: 16-bit hidden-layer rows (rpc_perturber_cfg.act16: 2 = bf16 gradient rows, 1 / 3 =
        # fp16 pre-activations / both). Off by default: measured r06 (profiles/r06_pert_act16_ab.txt) act16 = 2
        # takes the perturber backward 0.51 -> 0.435 ms (+0.5 % step) but moves the 6-step adversary update
        # cosine vs fp32 to 0.9949 and act16 = 3 to 0.9940, under tests/test_gpu_bf16_trajectory.py's 0.995
        adv.act16 = int(os.environ.get("RPC_PERT_ACT16", "0")) if bf16 else 0
    model.__dict__["_engine_mode"] = bool(bf16)
    if pin:
        model.__dict__["_engine_pinned"] = True


def _autocast_on() -> bool:
    try:
        return torch.is_autocast_enabled("cuda")
    except TypeError:   # older torch: no device argument
        return torch.is_autocast_enabled()


class DetectorBase(nn.Module):
    """forward(mode=) / train_step / val_step / test_step / parse_losses of mmengine BaseModel."""

    # ------------------------------------------------------------------ engines
    def _sync_engines(self, device: torch.device) -> None:
        """Follow the autocast state with the engines: bf16 (perf mode) under autocast, fp32 (parity mode)
        outside it — unless an engine mode was selected explicitly (Trainer / select_engines(pin=True)):
        then that mode stays, so val_step / test_step run on the engines the model trains on. A switch
        allocates the other engine's HIP graphs and dense BEV buffers on first use (the sparse encoder keeps
        only the current shapes' buffers); switching back to fp32 keeps the channels_last layout of the
        non-HIP modules (results are layout-independent)."""
        if device.type != "cuda" or self.__dict__.get("_engine_pinned"):
            return
        want = _autocast_on()
        if self.__dict__.get("_engine_mode") != want:
            select_engines(self, want)

    # ------------------------------------------------------------------ mmengine BaseModel
    def forward(self, inputs=None, data_samples=None, mode: str = "tensor", **kwargs):
        if mode == "loss":
            return self.loss(inputs, data_samples, **kwargs)
        if mode == "predict":
            return self.predict(inputs, data_samples, **kwargs)
        if mode == "tensor":
            return self._forward(inputs, data_samples, **kwargs)
        raise RuntimeError(f'Invalid mode "{mode}". Only supports loss, predict and tensor mode')

    def _forward(self, inputs, data_samples=None, **kwargs):
        """mmdet3d SingleStage3DDetector._forward: the head's raw outputs."""
        return self.bbox_head(self.extract_feat(inputs))

    def _run_forward(self, data, mode: str):
        if isinstance(data, dict):
            return self(**data, mode=mode)
        if isinstance(data, (list, tuple)):
            return self(*data, mode=mode)
        raise TypeError(f"Output of data_preprocessor should be a list, tuple or dict, got {type(data)}")

    def parse_losses(self, losses: dict):
        """mmengine BaseModel.parse_losses: (sum of every 'loss' key's mean(s), log_vars)."""
        return parse_losses(losses)

    def train_step(self, data, optim_wrapper):
        with optim_wrapper.optim_context(self):
            data = self.data_preprocessor(data, True)
            losses = self._run_forward(data, mode="loss")
        parsed, log_vars = self.parse_losses(losses)
        optim_wrapper.update_params(parsed)
        return log_vars

    @torch.no_grad()
    def val_step(self, data):
        data = self.data_preprocessor(data, False)
        return self._run_forward(data, mode="predict")

    @torch.no_grad()
    def test_step(self, data):
        data = self.data_preprocessor(data, False)
        return self._run_forward(data, mode="predict")


def ddp_train_step(ddp: nn.Module, data, optim_wrapper):
    """mmengine MMDistributedDataParallel.train_step: the forward goes through the DDP wrapper so
    its reducer sees the graph and all-reduces the gradient buckets during backward."""
    module = ddp.module
    with optim_wrapper.optim_context(ddp):
        data = module.data_preprocessor(data, True)
        losses = ddp(**data, mode="loss") if isinstance(data, dict) else ddp(*data, mode="loss")
    parsed, log_vars = module.parse_losses(losses)
    optim_wrapper.update_params(parsed)
    return log_vars


def det3d_gt(samples) -> Optional[tuple]:
    """(bboxes [Mi, K] tensors, labels [Mi] tensors) from mmdet3d Det3DDataSample-shaped samples,
    duck-typed: `sample.gt_instances_3d.bboxes_3d` (a LiDARInstance3DBoxes with `.tensor`, or a
    tensor) and `.labels_3d`; dict-style samples / instances are accepted too. None if `samples`
    is not such a list."""
    if not isinstance(samples, (list, tuple)) or not samples:
        return None
    first = samples[0]
    inst = lambda s: s.gt_instances_3d if hasattr(s, "gt_instances_3d") else \
        (s.get("gt_instances_3d") if isinstance(s, dict) else None)
    if inst(first) is None:
        return None
    boxes, labels = [], []
    for s in samples:
        g = inst(s)
        b = g.bboxes_3d if hasattr(g, "bboxes_3d") else g["bboxes_3d"]
        l = g.labels_3d if hasattr(g, "labels_3d") else g["labels_3d"]
        boxes.append(getattr(b, "tensor", b))
        labels.append(l)
    return boxes, labels
