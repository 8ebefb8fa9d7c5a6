"""a10: the reference's param_scheduler (configs/adversarial/…-3class.py:142-159) — mmengine
LinearLR(start_factor 0.1, end 2000 iters) chained with CosineAnnealingLR(T_max 30 epochs, eta_min
1e-6, convert_to_iter_based) — checked against mmengine's closed forms:

  LinearLR:           base * (s + (1 - s) * min(t, end - 1) / (end - 1))
  CosineAnnealingLR:  eta_min + (base - eta_min) * (1 + cos(pi * t / T)) / 2

(mmengine is not installed here; these are the `_get_closed_form_lr` formulas of its
LinearParamScheduler / CosineAnnealingParamScheduler). eta_min is one absolute floor for every
parameter group, and a hook's manual lr cut persists through later steps (the schedulers are
recursive)."""
import math

import pytest
import torch

from robustpointclouds_amd.trainer import LRSchedule, param_groups


class _Opt:
    def __init__(self, base=1e-4):
        m = torch.nn.Module()
        m.backbone = torch.nn.Linear(2, 2)
        m.adversary = torch.nn.Linear(2, 2)
        self.param_groups = param_groups(m, base)   # lr_mult 2.0 for 'adversary'


def _lin(t, s, end):
    return s + (1 - s) * min(t, end - 1) / (end - 1)


def _cos(t, b, eta, T):
    return eta + (b - eta) * (1 + math.cos(math.pi * t / T)) / 2


def test_groups_lr_mult():
    o = _Opt()
    assert [g["lr"] for g in o.param_groups] == pytest.approx([1e-4, 2e-4])


@pytest.mark.parametrize("ipe", [7, 50])
def test_linear_times_cosine_closed_form_without_floor(ipe):
    # eta_min = 0: the chained recursion is exactly the product of the two closed forms
    o = _Opt()
    warm = 40
    s = LRSchedule(o, iters_per_epoch=ipe, warmup=warm, T_max=3, eta_min=0.0)
    T = 3 * ipe
    for t in range(T):
        for g, b in zip(o.param_groups, s.base):
            want = b * _lin(t, 0.1, warm) * (1 + math.cos(math.pi * t / T)) / 2
            assert g["lr"] == pytest.approx(want, rel=1e-9, abs=1e-18), (t, b)
        s.step()


def test_cosine_absolute_eta_min_every_group():
    o = _Opt()
    s = LRSchedule(o, iters_per_epoch=10, warmup=0, T_max=30, eta_min=1e-6)
    T = 300
    for t in range(T):
        for g, b in zip(o.param_groups, s.base):
            assert g["lr"] == pytest.approx(_cos(t, b, 1e-6, T), rel=1e-9), (t, b)
        s.step()
    # both groups anneal to the same absolute floor (not eta_min * lr_mult)
    for g in o.param_groups:
        assert g["lr"] == pytest.approx(1e-6, rel=1e-2)


def test_warmup_start_and_end_values():
    o = _Opt()
    s = LRSchedule(o, iters_per_epoch=1000, warmup=2000, T_max=30, eta_min=1e-6)
    assert [g["lr"] for g in o.param_groups] == pytest.approx([1e-5, 2e-5])
    for _ in range(1999):
        s.step()
    T = 30000
    for g, b in zip(o.param_groups, s.base):
        # the linear factor has reached 1; cosine has moved 1999 of 30000 steps (floor term within 1e-3)
        assert g["lr"] == pytest.approx(_cos(1999, b, 1e-6, T), rel=1e-3)


def test_hook_lr_cut_persists():
    a, b = _Opt(), _Opt()
    sa = LRSchedule(a, iters_per_epoch=5, warmup=20, T_max=30, eta_min=0.0)
    sb = LRSchedule(b, iters_per_epoch=5, warmup=20, T_max=30, eta_min=0.0)
    for t in range(10):
        sa.step()
        sb.step()
    for g in b.param_groups:        # NaNDetectionHook: g['lr'] *= 0.1
        g["lr"] *= 0.1
    for t in range(25):
        sa.step()
        sb.step()
        for ga, gb in zip(a.param_groups, b.param_groups):
            assert gb["lr"] == pytest.approx(0.1 * ga["lr"], rel=1e-9)


def test_nan_hook_cut_then_schedule():
    """NaNDetectionHook (custom_hook.py:94-151) cuts lr x0.1 after max_nan_count NaN steps; the next
    scheduler steps rescale from the cut value (mmengine order: hook, then ParamSchedulerHook)."""
    from types import SimpleNamespace

    from robustpointclouds_amd.plugin.custom_hook import NaNDetectionHook
    a, b = _Opt(), _Opt()
    sa = LRSchedule(a, iters_per_epoch=5, warmup=20, T_max=30, eta_min=0.0)
    sb = LRSchedule(b, iters_per_epoch=5, warmup=20, T_max=30, eta_min=0.0)
    runner = SimpleNamespace(optim_wrapper=SimpleNamespace(optimizer=b), model=torch.nn.Module(), should_stop=False)
    hook = NaNDetectionHook(max_nan_count=3)
    nan = dict(loss_cls=torch.tensor(float("nan")), loss_bbox=torch.tensor(1.0), perturbation_l2_norm=torch.tensor(0.1))
    for i in range(3):
        hook.after_train_iter(runner, i, None, nan)
        sa.step()
        sb.step()
    assert hook.lr_reduced
    for _ in range(5):
        hook.after_train_iter(runner, 0, None, dict(loss_cls=torch.tensor(0.5)))
        sa.step()
        sb.step()
        for ga, gb in zip(a.param_groups, b.param_groups):
            assert gb["lr"] == pytest.approx(0.1 * ga["lr"], rel=1e-9)
