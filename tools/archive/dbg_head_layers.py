"""Debug: record every ConvModule backward the fp32 HIP CenterHead issues and recompute each one in float64
from the recorded fp32 inputs (h, dh, weights, BN batch statistics)."""
import sys

import torch
import torch.nn.functional as Fn

sys.path.insert(0, ".")
from robustpointclouds_amd import center_head as ch  # noqa: E402
from robustpointclouds_amd import dense_bev as db  # noqa: E402
from robustpointclouds_amd.center_head import _BOX_ORDER, CenterHead  # noqa: E402

DEV = torch.device("cuda")
rel = lambda a, b: float((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30))
REC = []
orig = db._backward_layer


def spy(eng, rec, dh, dh_pitch, dh_off, dev, st, need_dx, dx_out=None, accumulate=False, bn_part=None, next_rec=None):
    dh_copy = dh.clone()
    base = dx_out.clone() if (dx_out is not None and accumulate) else None
    out = orig(eng, rec, dh, dh_pitch, dh_off, dev, st, need_dx, dx_out, accumulate, bn_part, next_rec)
    torch.cuda.synchronize()
    REC.append(dict(L=rec["L"], h=rec["h"].clone(), dh=dh_copy, out=[o.clone() if o is not None else None for o in out[:4]],
                    base=base))
    return out


ch.db._backward_layer = spy

torch.manual_seed(0)
B, H = 2, 32
head = CenterHead(in_channels=128).to(DEV)
with torch.no_grad():
    for th in head.task_heads:
        for dcn in (th.feature_adapt_cls, th.feature_adapt_reg):
            dcn.conv_offset.weight.normal_(0, 0.02)
            dcn.conv_offset.bias.uniform_(-0.5, 0.5)
x = torch.randn(B, 128, H, H)
g = torch.Generator().manual_seed(5)
ghm = torch.zeros(B, 10, H, H)
gbox = torch.zeros(B, 60, H, H)
gbox[:, 10:12] = torch.randn(B, 2, H, H, generator=g)
xd = x.to(DEV).requires_grad_(True)
preds = head([xd])
hm = torch.cat([p[0]["heatmap"] for p in preds], 1)
box = torch.cat([torch.cat([p[0][n] for n in _BOX_ORDER], 1) for p in preds], 1)
((hm * ghm.to(DEV)).sum() + (box * gbox.to(DEV)).sum()).backward()
torch.cuda.synchronize()
for i, r in enumerate(REC):
    L = r["L"]
    if float(r["dh"].abs().max()) == 0.0:
        continue
    h = r["h"].double().cpu().requires_grad_(True)
    W = L.conv.weight.detach().double().cpu().requires_grad_(True)
    gm = L.bnm.weight.detach().double().cpu().requires_grad_(True)
    bt = L.bnm.bias.detach().double().cpu().requires_grad_(True)
    z = Fn.conv2d(h, W, padding=1)
    m = z.mean((0, 2, 3), keepdim=True)
    v = z.var((0, 2, 3), unbiased=False, keepdim=True)
    y = torch.relu((z - m) / torch.sqrt(v + L.bnm.eps) * gm.view(1, -1, 1, 1) + bt.view(1, -1, 1, 1))
    (y * r["dh"].double().cpu()).sum().backward()
    dx, dW, dg, dbeta = r["out"]
    if r["base"] is not None:
        dx = dx - r["base"]
    pre = ((z - m) / torch.sqrt(v + L.bnm.eps) * gm.view(1, -1, 1, 1) + bt.view(1, -1, 1, 1)).detach()
    near = int((pre.abs() < 1e-5).sum())
    print(f"{i:2d} {tuple(L.conv.weight.shape)} dh max {float(r['dh'].abs().max()):.2e}: dx {rel(dx.cpu(), h.grad):.2e} "
          f"dW {rel(dW.cpu(), W.grad):.2e} dgamma {rel(dg.cpu(), gm.grad):.2e} dbeta {rel(dbeta.cpu(), bt.grad):.2e} "
          f"(|pre| < 1e-5: {near})")

# the recorded dh of task 1's reg.0 ConvModule against the float64 data gradient of its final conv
fc = head.task_heads[1].task_head.reg[1]
dz = gbox[:, 10:12].double()
hr_shape = REC[7]["dh"].shape
zin = torch.zeros(hr_shape, dtype=torch.float64, requires_grad=True)
out = Fn.conv2d(zin, fc.weight.detach().double().cpu(), None, padding=1)
(out * dz).sum().backward()
dh_ref = zin.grad
dh_hip = REC[7]["dh"].double().cpu()
print("final-conv dgrad: dh rel", rel(dh_hip, dh_ref), "max abs", float((dh_hip - dh_ref).abs().max()),
      "ref max", float(dh_ref.abs().max()))
err = (dh_hip - dh_ref).abs()
idx = (err > 1e-3 * float(dh_ref.abs().max())).nonzero()
print("elements off:", idx.shape[0], idx[:10].tolist())
