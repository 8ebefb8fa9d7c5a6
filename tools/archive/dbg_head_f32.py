"""Debug: fp32 HIP CenterHead vs the float64 torch stack at CenterPoint's BEV size, sparse / dense input."""
import sys

import torch

sys.path.insert(0, ".")
from tests.test_gpu_dcn_head import _ref_head  # noqa: E402
from tests.test_gpu_e2e_parity_centerpoint import _CenterHead  # noqa: E402
from robustpointclouds_amd.center_head import _BOX_ORDER, CenterHead  # noqa: E402

DEV = torch.device("cuda")


def run(B, H, W, sparse, seed=0, cin=128, only=None):
    torch.manual_seed(seed)
    head = CenterHead(in_channels=cin).to(DEV)
    with torch.no_grad():
        for th in head.task_heads:
            for dcn in (th.feature_adapt_cls, th.feature_adapt_reg):
                dcn.conv_offset.weight.normal_(0, 0.02)
                dcn.conv_offset.bias.uniform_(-0.5, 0.5)
    x = torch.randn(B, cin, H, W)
    if sparse:
        m = (torch.rand(B, 1, H, W) < 0.15).float()
        x = x * m
    xd = x.to(DEV).requires_grad_(True)
    preds = head([xd])
    hm = torch.cat([p[0]["heatmap"] for p in preds], 1)
    box = torch.cat([torch.cat([p[0][n] for n in _BOX_ORDER], 1) for p in preds], 1)
    g = torch.Generator().manual_seed(5)
    ghm, gbox = torch.randn(hm.shape, generator=g).double(), torch.randn(box.shape, generator=g).double()
    if only == "hm":
        gbox.zero_()
    elif only is not None:     # one box channel range only
        keep = torch.zeros_like(gbox)
        keep[:, only[0]:only[1]] = gbox[:, only[0]:only[1]]
        gbox = keep
        ghm.zero_()
    ((hm * ghm.float().to(DEV)).sum() + (box * gbox.float().to(DEV)).sum()).backward()
    ref = _CenterHead(head, torch.float64)
    xr = x.double().requires_grad_(True)
    rh, rb = ref([xr])
    ((torch.cat(rh, 1) * ghm).sum() + (torch.cat(rb, 1) * gbox).sum()).backward()
    r32 = _CenterHead(head, torch.float32)
    x32 = x.float().requires_grad_(True)
    sh, sb = r32([x32])
    ((torch.cat(sh, 1) * ghm.float()).sum() + (torch.cat(sb, 1) * gbox.float()).sum()).backward()
    p32 = dict(r32.m.named_parameters())
    rel = lambda a, b: float((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30))
    out = [(rel(xd.grad.cpu(), xr.grad), "x", rel(x32.grad, xr.grad))]
    rp = dict(ref.m.named_parameters())
    for n, p in head.named_parameters():
        out.append((rel(p.grad.cpu(), rp[n].grad), n, rel(p32[n].grad, rp[n].grad)))
    out.sort(reverse=True)
    print(f"B={B} {H}x{W} sparse={sparse} only={only}: fwd hm {rel(hm.detach().cpu(), torch.cat(rh, 1).detach()):.2e}")
    rbx = torch.cat(rb, 1).detach()
    print("   box fwd per channel:", " ".join(f"{c}:{rel(box.detach().cpu()[:, c], rbx[:, c]):.1e}" for c in range(rbx.shape[1])))
    for e, n, e32 in out[:8]:
        print(f"   hip {e:.3e}  torch-cpu-fp32 {e32:.3e}  {n}")


for only in ((10, 12),):
    run(2, 32, 32, False, only=only)
