"""Mirror of /root/reference/custom_hook.py: EpochTrackerHook (:18-75), NaNDetectionHook
(:77-151) and the no-op L2NormRegularizationHook (:5-16), registered into mmengine HOOKS
when installed. They also work with robustpointclouds_amd.trainer.Trainer (same runner
attributes: model, epoch, optim_wrapper, should_stop, logger)."""
import logging

import torch

try:
    from mmengine.hooks import Hook
    from mmengine.registry import HOOKS
except ImportError:   # standalone
    class Hook:  # noqa: D401 - minimal stand-in
        """Base hook."""

    HOOKS = None


def _reg(cls):
    from robustpointclouds_amd.registry import HOOKS as _LOCAL_HOOKS
    _LOCAL_HOOKS.register_module(module=cls)   # custom_hooks=[dict(type=...)] without mmengine
    if HOOKS is not None:
        HOOKS.register_module(module=cls, force=True)
    return cls


def _inner(model):
    return model.module if hasattr(model, "module") else model


@_reg
class L2NormRegularizationHook(Hook):
    """Defines no hook methods in the reference (:5-16): a no-op."""

    def __init__(self, regularization_strength=0.01):
        self.regularization_strength = regularization_strength


@_reg
class EpochTrackerHook(Hook):
    """Sets model._epoch before every train/val epoch (:22-28, :42-48). The reference's first
    after_train_iter (:30-40) is shadowed by the second (:50-75), which never fires because
    the outputs carry no 'l2_norm' key; neither is reproduced."""

    def before_train_epoch(self, runner):
        _inner(runner.model)._epoch = runner.epoch

    def before_val_epoch(self, runner):
        _inner(runner.model)._epoch = runner.epoch


@_reg
class NaNDetectionHook(Hook):
    """:77-151 — NaN/Inf loss watchdog: LR x0.1 after max_nan_count, stop after 50 in a row,
    reset adversary weights, disable the adversary after 100 in total."""

    def __init__(self, max_nan_count=10):
        self.max_nan_count = max_nan_count
        self.nan_count = 0
        self.lr_reduced = False
        self.consecutive_nan_count = 0
        self.total_nan_count = 0

    def after_train_iter(self, runner, batch_idx, data_batch=None, outputs=None):
        log = getattr(runner, "logger", logging.getLogger("rpc"))
        outputs = outputs or {}
        keys = [k for k, v in outputs.items() if "loss" in k and isinstance(v, torch.Tensor)]
        bad = []
        if keys:   # one device->host read for all loss keys (not one sync per key)
            fin = torch.stack([torch.isfinite(outputs[k]).all() for k in keys]).cpu()
            bad = [k for k, ok in zip(keys, fin.tolist()) if not ok]
        if bad:
            self.nan_count += 1
            self.consecutive_nan_count += 1
            self.total_nan_count += 1
            log.warning(f"NaN/Inf in {bad}; count {self.nan_count}/{self.max_nan_count}")
            if self.consecutive_nan_count >= 50:
                runner.should_stop = True
                return
            if self.nan_count >= self.max_nan_count and not self.lr_reduced:
                for g in runner.optim_wrapper.optimizer.param_groups:
                    g["lr"] *= 0.1
                self.lr_reduced = True
                self.nan_count = 0
                model = _inner(runner.model)
                if getattr(model, "adversary", None) is not None:
                    model.adversary._reset_problematic_weights()
                if self.total_nan_count > 100 and hasattr(model, "disable_adversarial_training"):
                    model.disable_adversarial_training()
        else:
            self.consecutive_nan_count = 0
            self.nan_count = max(0, self.nan_count - 1)
