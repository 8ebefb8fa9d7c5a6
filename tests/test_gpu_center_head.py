"""§8(f3): CenterHead targets + losses on the HIP kernels (csrc/center_head.hip) vs the CPU
restatement oracle/center_head.py on the same head outputs.

Targets: ind / mask exact, the gaussian target heatmap exact (float64 gaussian cast to float32 on
both sides), anno boxes within 1e-6 (device log/sin/cos vs the host's). Losses within 1e-5 relative
(fp32 sums in a different order), d loss / d logits and d loss / d boxes within 1e-4 relative-L2 of
torch autograd through the oracle. Parity w.r.t. upstream mmdet3d is unpinned (not vendored)."""
import ctypes as C

import pytest
import torch

from oracle import center_head as oc
from robustpointclouds_amd import _ffi
from robustpointclouds_amd.center_head import (NUS_TASKS, NUS_TRAIN_CFG, CenterLossFn, center_cfg, center_targets,
                                               pack_gt)
from tests._center_data import nus_gts

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


def _setup(B, seed, max_objs=500, n=30, H=128, W=128, empty=()):
    tc = dict(NUS_TRAIN_CFG, max_objs=max_objs)
    ocfg = oc.CenterCfg(max_objs=max_objs, grid_size=(W * 8, H * 8, 40))
    tc["grid_size"] = [W * 8, H * 8, 40]
    N = sum(len(t) for t in NUS_TASKS)
    cfg = center_cfg(NUS_TASKS, tc, B, H, W, hm_pitch=N + 2, box_pitch=60 + 4)
    gts = nus_gts(B, seed, n=n)
    gts = [(b[:0], l[:0]) if i in empty else (b, l) for i, (b, l) in enumerate(gts)]
    g = torch.Generator().manual_seed(seed)
    hm = torch.randn(B * H * W, N + 2, generator=g) * 2.0
    box = torch.randn(B * H * W, 64, generator=g)
    return cfg, ocfg, gts, hm, box


def _oracle_inputs(hm, box, B, H, W):
    T = len(NUS_TASKS)
    hm4 = hm.view(B, H, W, -1)
    bx4 = box.view(B, H, W, -1)
    hl, bl, c0 = [], [], 0
    for t, names in enumerate(NUS_TASKS):
        hl.append(hm4[..., c0:c0 + len(names)].permute(0, 3, 1, 2))
        bl.append(bx4[..., 10 * t:10 * t + 10].permute(0, 3, 1, 2))
        c0 += len(names)
    return hl, bl, T


@pytest.mark.parametrize("seed,max_objs,empty", [(1, 500, ()), (2, 4, ()), (3, 500, (1,))])
def test_targets_exact(seed, max_objs, empty):
    B, H, W = 2, 128, 128
    cfg, ocfg, gts, hm, box = _setup(B, seed, max_objs, empty=empty)
    gb, gl = pack_gt([b for b, _ in gts], [l for _, l in gts], DEV)
    lib = _ffi.load()
    wsz = lib.rpc_center_head_workspace_size(C.byref(cfg), gl.shape[1])
    ws = torch.empty(wsz, dtype=torch.uint8, device=DEV)
    out = torch.empty(12, device=DEV)
    hmd, bxd = hm.to(DEV), box.to(DEV)
    _ffi.check(lib.rpc_center_head_loss_forward(C.byref(cfg), _ffi.ptr(gb), _ffi.ptr(gl), gl.shape[1], _ffi.ptr(hmd),
                                                _ffi.ptr(bxd), _ffi.ptr(out), _ffi.ptr(ws), wsz,
                                                _ffi.stream_of(hmd)), "fwd")
    th, ti, tm, ta = [t.cpu() for t in center_targets(cfg, ws, gl.shape[1])]
    hms, annos, inds, masks = oc.targets(ocfg, [b for b, _ in gts], [l for _, l in gts])
    c0 = 0
    for t, names in enumerate(NUS_TASKS):
        want = hms[t].permute(0, 2, 3, 1)
        assert torch.equal(th[..., c0:c0 + len(names)], want), f"task {t} heatmap"
        c0 += len(names)
        assert torch.equal(tm[:, t].long(), masks[t].long()), f"task {t} mask"
        assert torch.equal(ti[:, t].long() * tm[:, t].long(), inds[t] * masks[t].long()), f"task {t} ind"
        torch.testing.assert_close(ta[:, t], annos[t], rtol=0, atol=2e-6)


@pytest.mark.parametrize("seed,max_objs,empty", [(4, 500, ()), (5, 3, ()), (6, 500, (0, 1))])
def test_losses_and_grads(seed, max_objs, empty):
    B, H, W = 2, 128, 128
    cfg, ocfg, gts, hm, box = _setup(B, seed, max_objs, empty=empty)
    gb, gl = pack_gt([b for b, _ in gts], [l for _, l in gts], DEV)
    hmd = hm.to(DEV).requires_grad_(True)
    bxd = box.to(DEV).requires_grad_(True)
    out = CenterLossFn.apply(hmd, bxd, gb, gl, cfg)
    w = torch.linspace(0.5, 1.5, out.numel(), device=DEV)
    (out * w).sum().backward()
    hmo = hm.clone().double().requires_grad_(True)
    bxo = box.clone().double().requires_grad_(True)
    hl, bl, T = _oracle_inputs(hmo, bxo, B, H, W)
    ref = oc.losses(ocfg, hl, bl, [b for b, _ in gts], [l for _, l in gts])
    refv = torch.stack([ref[f"task{t}.{k}"] for t in range(T) for k in ("loss_heatmap", "loss_bbox")])
    torch.testing.assert_close(out.detach().cpu().double(), refv.detach(), rtol=1e-5, atol=1e-7)
    (refv * w.cpu().double()).sum().backward()
    for got, want, name in ((hmd.grad, hmo.grad, "dhm"), (bxd.grad, bxo.grad, "dbox")):
        g, r = got.cpu().double(), want
        N = sum(len(t) for t in NUS_TASKS)
        cols = slice(0, N) if name == "dhm" else slice(0, 60)
        err = (g[:, cols] - r[:, cols]).norm() / max(r[:, cols].norm().item(), 1e-30)
        assert err < 1e-4, f"{name} rel-L2 {err:.2e}"


def test_deterministic():
    B, H, W = 2, 128, 128
    cfg, _, gts, hm, box = _setup(B, 7)
    gb, gl = pack_gt([b for b, _ in gts], [l for _, l in gts], DEV)
    outs = [CenterLossFn.apply(hm.to(DEV), box.to(DEV), gb, gl, cfg) for _ in range(2)]
    assert torch.equal(outs[0], outs[1])
