"""Debug: is the fp32 HIP CenterHead backward run-to-run deterministic? (per-parameter max |diff|)"""
import sys

import torch

sys.path.insert(0, ".")
from robustpointclouds_amd.center_head import _BOX_ORDER, CenterHead  # noqa: E402

DEV = torch.device("cuda")


def step(head, x, ghm, gbox, dt):
    head.zero_grad(set_to_none=True)
    xd = x.to(DEV).to(dt).requires_grad_(True)
    preds = head([xd])
    hm = torch.cat([p[0]["heatmap"] for p in preds], 1)
    box = torch.cat([torch.cat([p[0][n] for n in _BOX_ORDER], 1) for p in preds], 1)
    ((hm * ghm).sum() + (box * gbox).sum()).backward()
    torch.cuda.synchronize()
    return {n: p.grad.clone() for n, p in head.named_parameters()}, xd.grad.clone()


for dt in (torch.float32, torch.bfloat16):
    for B, H in ((2, 32), (2, 128)):
        torch.manual_seed(0)
        head = CenterHead(in_channels=128).to(DEV)
        with torch.no_grad():
            for th in head.task_heads:
                for dcn in (th.feature_adapt_cls, th.feature_adapt_reg):
                    dcn.conv_offset.weight.normal_(0, 0.02)
                    dcn.conv_offset.bias.uniform_(-0.5, 0.5)
        x = torch.randn(B, 128, H, H)
        g = torch.Generator().manual_seed(5)
        ghm = torch.randn(B, 10, H, H, generator=g).to(DEV)
        gbox = torch.randn(B, 60, H, H, generator=g).to(DEV)
        a, ax = step(head, x, ghm, gbox, dt)
        b, bx = step(head, x, ghm, gbox, dt)
        diffs = sorted(((float((a[n] - b[n]).abs().max()) / max(float(a[n].abs().max()), 1e-30), n) for n in a),
                       reverse=True)
        print(f"{dt} B={B} {H}x{H}: x max rel diff {float((ax - bx).abs().max()) / float(ax.abs().max()):.2e}; "
              f"params differing: {sum(d > 0 for d, _ in diffs)} of {len(diffs)}; worst {diffs[:4]}")
