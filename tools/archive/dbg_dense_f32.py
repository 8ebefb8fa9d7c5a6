"""Debug: fp32 dense engine pieces the CenterHead uses (3x3 S1 conv 64->64 fwd / dgrad / wgrad, no BN;
ConvModule fwd/bwd) vs float64 torch, at the head's sizes."""
import sys

import torch
import torch.nn.functional as Fn

sys.path.insert(0, ".")
from robustpointclouds_amd import _ffi  # noqa: E402
from robustpointclouds_amd import dense_bev as db  # noqa: E402
from robustpointclouds_amd.center_head import _conv_nobn_bwd, _conv_nobn_fwd, _conv_module_layer, ConvModule  # noqa: E402

DEV = torch.device("cuda")
rel = lambda a, b: float((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30))


def nobn(B, H, W, ci, co):
    torch.manual_seed(1)
    lib = _ffi.load()
    eng = db._Eng(lib, True)
    st = _ffi.stream_of(torch.empty(1, device=DEV))
    x = torch.randn(B, ci, H, W)
    w = torch.randn(co, ci, 3, 3) * 0.05
    g = torch.randn(B, co, H, W)
    xi = db._nhwc(x.to(DEV), torch.float32)
    z, rec = _conv_nobn_fwd(eng, w.to(DEV), ci, xi, ci, B, H, W, DEV, st)
    dz = db._nhwc(torch.cat([g, torch.zeros(B, 64 - co, H, W)], 1).to(DEV), torch.float32)
    dx, dW = _conv_nobn_bwd(eng, rec, dz, DEV, st)
    torch.cuda.synchronize()
    xr = x.double().requires_grad_(True)
    wr = w.double().requires_grad_(True)
    zr = Fn.conv2d(xr, wr, padding=1)
    (zr * g.double()).sum().backward()
    print(f"nobn B={B} {H}x{W} {ci}->{co}: z {rel(z[:, :co].cpu(), zr.detach()):.2e} "
          f"dx {rel(dx.cpu(), xr.grad):.2e} dW {rel(dW.cpu(), wr.grad):.2e}")


def convmodule(B, H, W, ci, co):
    torch.manual_seed(2)
    lib = _ffi.load()
    eng = db._Eng(lib, True)
    st = _ffi.stream_of(torch.empty(1, device=DEV))
    cm = ConvModule(ci, co).to(DEV).train()
    with torch.no_grad():
        cm.bn.weight.uniform_(0.5, 1.5)
        cm.bn.bias.uniform_(-0.2, 0.2)
    x = torch.randn(B, ci, H, W)
    g = torch.randn(B, co, H, W)
    L = _conv_module_layer(cm)
    xi = db._nhwc(x.to(DEV), torch.float32)
    y, rec, _, _ = db._forward_layer(eng, L, xi, ci, B, H, W, True, DEV, st)
    gi = db._nhwc(g.to(DEV), torch.float32)
    dx, dWc, dg, dbt, _ = db._backward_layer(eng, rec, gi, co, 0, DEV, st, True)
    torch.cuda.synchronize()
    xr = x.double().requires_grad_(True)
    P = {k: v.detach().cpu().double().requires_grad_(True) for k, v in cm.named_parameters()}
    z = Fn.conv2d(xr, P["conv.weight"], padding=1)
    m = z.mean((0, 2, 3), keepdim=True)
    v = z.var((0, 2, 3), unbiased=False, keepdim=True)
    yr = torch.relu((z - m) / torch.sqrt(v + cm.bn.eps) * P["bn.weight"].view(1, -1, 1, 1) + P["bn.bias"].view(1, -1, 1, 1))
    (yr * g.double()).sum().backward()
    print(f"convmodule B={B} {H}x{W} {ci}->{co}: y {rel(y.cpu(), yr.detach()):.2e} dx {rel(dx.cpu(), xr.grad):.2e} "
          f"dW {rel(dWc.cpu(), P['conv.weight'].grad):.2e} dgamma {rel(dg.cpu(), P['bn.weight'].grad):.2e} "
          f"dbeta {rel(dbt.cpu(), P['bn.bias'].grad):.2e}")


for shp in [(2, 32, 32), (2, 128, 128), (1, 16, 16)]:
    nobn(*shp, 64, 64)
    nobn(*shp, 64, 2)
    convmodule(*shp, 64, 64)
    convmodule(*shp, 128, 64)
