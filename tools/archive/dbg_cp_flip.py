"""Which discrete decisions flip between the float64 oracle step and the same step fed HIP's neck output (N_hip)
or the fp32 oracle's (N32)? Records every ReLU mask of the backbone / neck / CenterHead stack and every DCN
sample's bilinear cell (floor of the sampling position) and validity, per layer in call order, and counts the
entries that differ from the plain float64 run (tests/test_gpu_e2e_parity_centerpoint.py setup)."""
import sys

B = 2   # the r04 case: frames() defaults (2 one-sweep frames)

import torch
from torch import nn

sys.path.insert(0, ".")
import oracle.dcn as odcn  # noqa: E402
import tests.test_gpu_e2e_parity_centerpoint as tp  # noqa: E402
from tests.test_gpu_e2e_parity_centerpoint import OracleStep, frames, oracle_voxels  # noqa: E402
from robustpointclouds_amd.adversarial_loss import parse_losses  # noqa: E402
from robustpointclouds_amd.center_head import pack_gt  # noqa: E402
from robustpointclouds_amd.trainer import Trainer, make_nus_model  # noqa: E402

REC = None   # list of (tag, tensor) of the current oracle run


def rec(tag, t):
    if REC is not None:
        REC.append((tag, t.detach().clone()))


_orig_cm = tp._CenterHead._cm


def cm(cmod, h):
    z = tp.Fn.conv2d(h, cmod.conv.weight, padding=1)
    m = z.mean((0, 2, 3), keepdim=True)
    v = z.var((0, 2, 3), unbiased=False, keepdim=True)
    pre = (z - m) / torch.sqrt(v + cmod.bn.eps) * cmod.bn.weight.view(1, -1, 1, 1) + cmod.bn.bias.view(1, -1, 1, 1)
    rec("head.relu", pre)
    return torch.relu(pre)


tp._CenterHead._cm = staticmethod(cm)
_orig_dcn = odcn.deform_conv2d


def dcn(x, offset, weight, groups=4):
    rec("dcn.offset", offset)
    return _orig_dcn(x, offset, weight, groups)


tp.deform_conv2d = dcn


def hook_relus(mod, name):
    for n, m in mod.named_modules():
        if isinstance(m, nn.ReLU):
            m.register_forward_pre_hook(lambda mm, inp, n=n: rec(f"{name}.{n}", inp[0]))


def subst(sub):
    def hook(mod, inp, out):
        t = out[0]
        s = t.detach().clone()
        s.copy_(sub.to(dtype=t.dtype).view_as(t))
        return [t + (s - t).detach()]
    return hook


def run_oracle(model, dtype, subN=None, cap=None):
    global REC
    o = OracleStep(model, dtype)
    hook_relus(o.ref.pts_backbone, "backbone")
    hook_relus(o.ref.pts_neck, "neck")
    if subN is not None:
        o.ref.pts_neck.register_forward_hook(subst(subN))
    if cap is not None:
        o.ref.pts_neck.register_forward_hook(lambda m, i, out: cap.__setitem__("N", out[0].detach().clone()))
    REC = []
    o.step(rv, rn, rc, ogts)
    r, REC = REC, None
    return r


def frac_stats(off, H, W):
    """offset [B, 18, H, W] -> per tap the sampling positions; distance of each to the nearest integer"""
    ys = torch.arange(H, dtype=off.dtype).view(1, H, 1)
    xs = torch.arange(W, dtype=off.dtype).view(1, 1, W)
    d = []
    for k in range(9):
        i, j = k // 3, k % 3
        ph = ys - 1 + i + off[:, 2 * k]
        pw = xs - 1 + j + off[:, 2 * k + 1]
        d += [(ph - ph.round()).abs().flatten(), (pw - pw.round()).abs().flatten()]
    return torch.cat(d)


def compare(tag, a, b):
    print(f"== {tag}")
    for (ta, x), (tb, y) in zip(a, b):
        assert ta == tb
        if ta == "dcn.offset":
            H, W = x.shape[-2:]
            fl = lambda o: torch.cat([torch.floor(torch.arange(H, dtype=o.dtype).view(1, H, 1) - 1 + k // 3 + o[:, 2 * k]).flatten()
                                      for k in range(9)] + [torch.floor(torch.arange(W, dtype=o.dtype).view(1, 1, W) - 1 + k % 3
                                                                        + o[:, 2 * k + 1]).flatten() for k in range(9)])
            nd = int((fl(x) != fl(y)).sum())
            dist = frac_stats(x, H, W)
            print(f"  {ta:40s} cells differing {nd:8d} / {dist.numel()}; positions within 1e-6 / 1e-5 / 1e-4 of an "
                  f"integer: {int((dist < 1e-6).sum())} / {int((dist < 1e-5).sum())} / {int((dist < 1e-4).sum())}; "
                  f"offset rel diff {float((x - y).norm() / x.norm()):.2e}")
        else:
            mx, my = x > 0, y > 0
            nd = int((mx != my).sum())
            sc = x.abs().amax(dim=tuple(i for i in range(x.dim()) if i != 1), keepdim=True).clamp_min(1e-30)
            small = int(((x.abs() / sc) < 1e-6).sum())
            if nd or small:
                # per channel: the channels whose masks differ, and how many entries each
                per = (mx != my).sum(dim=tuple(i for i in range(x.dim()) if i != 1))
                worst = torch.topk(per.flatten(), min(3, per.numel()))
                print(f"  {ta:40s} mask differs at {nd:8d} of {x.numel()}; |pre| < 1e-6 max: {small}; "
                      f"worst channels {worst.indices.tolist()} ({worst.values.tolist()})")


dev = torch.device("cuda")
torch.manual_seed(21)
model = make_nus_model(device=dev, epoch=3)
with torch.no_grad():
    for th in model.pts_bbox_head.task_heads:
        for d in (th.feature_adapt_cls, th.feature_adapt_reg):
            d.conv_offset.weight.normal_(0, 0.02)
            d.conv_offset.bias.uniform_(-0.5, 0.5)
Trainer._select_engines(model, bf16=False)
model.train()
pts, gts = frames()
rv, rc, rn = oracle_voxels(pts)
ogts = dict(boxes=[torch.from_numpy(b) for b, _ in gts], labels=[torch.from_numpy(l) for _, l in gts])
gpts = [torch.from_numpy(p).to(dev) for p in pts]
gb, gl = pack_gt([torch.from_numpy(b) for b, _ in gts], [torch.from_numpy(l) for _, l in gts], dev)
cap = {}
model.pts_neck.register_forward_hook(lambda m, i, o: cap.__setitem__("N", o[0].detach().float().cpu()))
batch = model.data_preprocessor(dict(inputs=dict(points=gpts)), training=True)["inputs"]
batch["batch_size"] = B
losses = model.loss(batch, dict(gt_boxes=gb, gt_labels=gl))
torch.cuda.synchronize()
N_hip = cap["N"]
c32 = {}
run_oracle(model, torch.float32, cap=c32)
r64 = run_oracle(model, torch.float64)
r_hip = run_oracle(model, torch.float64, subN=N_hip)
r_32 = run_oracle(model, torch.float64, subN=c32["N"])
compare("f64 | N_hip vs f64", r64, r_hip)
compare("f64 | N32 vs f64", r64, r_32)
