import torch
from robustpointclouds_amd.second import SECOND, SECONDFPN
DEV = torch.device("cuda")

def mods(seed, ln):
    torch.manual_seed(seed)
    bb = SECOND(in_channels=256, layer_nums=ln, layer_strides=[1, 2], out_channels=[128, 256])
    nk = SECONDFPN(in_channels=[128, 256], upsample_strides=[1, 2], out_channels=[256, 256])
    for m in list(bb.modules()) + list(nk.modules()):
        if isinstance(m, torch.nn.BatchNorm2d):
            with torch.no_grad():
                m.weight.uniform_(0.5, 1.5); m.bias.uniform_(-0.2, 0.2)
    return bb.to(DEV), nk.to(DEV)

cos = lambda a, b: (a.flatten().double() @ b.flatten().double() / (a.double().norm() * b.double().norm())).item()
for ln in ([0, 0], [1, 1], [2, 2], [5, 5]):
    B, H, W = 2, 40, 36
    x = torch.relu(torch.randn(B, 256, H, W, generator=torch.Generator().manual_seed(5))).to(DEV)
    bbr, nkr = mods(0, ln); bb, nk = mods(0, ln); bb.hip = nk.hip = True
    # reference on bf16-rounded input in fp32
    xr = x.to(torch.bfloat16).float().requires_grad_(True)
    ref = nkr(bbr(xr))[0]
    xh = x.to(torch.bfloat16).contiguous(memory_format=torch.channels_last).requires_grad_(True)
    out = nk(bb(xh))[0]
    G = torch.randn(ref.shape, generator=torch.Generator().manual_seed(6)).to(DEV)
    (ref * G).sum().backward(); (out.float() * G).sum().backward()
    print(ln, "fwd rel", ((out.float() - ref).norm() / ref.norm()).item(), "dx cos", cos(xh.grad.float(), xr.grad))
    for (n, p), (_, q) in zip(list(bb.named_parameters()) + list(nk.named_parameters()),
                              list(bbr.named_parameters()) + list(nkr.named_parameters())):
        print("   ", n, round(cos(p.grad, q.grad), 5), "norm ratio", round((p.grad.norm() / q.grad.norm()).item(), 4))
