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
for ln in ([0, 0], [2, 2], [5, 5]):
    B, H, W = 2, 40, 36
    x = torch.relu(torch.randn(B, 256, H, W, generator=torch.Generator().manual_seed(5))).to(DEV)
    G = None
    res = {}
    for mode in ("fp32", "autocast", "hip"):
        bb, nk = mods(0, ln)
        if mode == "hip":
            bb.hip = nk.hip = True
        xi = x.to(torch.bfloat16).float()
        if mode != "fp32":
            bb.to(memory_format=torch.channels_last); nk.to(memory_format=torch.channels_last)
            xi = xi.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        xi = xi.requires_grad_(True)
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=(mode != "fp32")):
            out = nk(bb(xi))[0]
        if G is None:
            G = torch.randn(out.shape, generator=torch.Generator().manual_seed(6)).to(DEV)
        (out.float() * G).sum().backward()
        res[mode] = (out.detach().float(), xi.grad.float(), [p.grad.float() for p in list(bb.parameters()) + list(nk.parameters())])
    for mode in ("autocast", "hip"):
        o, gx, gp = res[mode]
        r = res["fp32"]
        cs = [cos(a, b) for a, b in zip(gp, r[2])]
        print(ln, mode, "fwd rel %.4f" % ((o - r[0]).norm() / r[0].norm()).item(), "dx cos %.5f" % cos(gx, r[1]),
              "param cos min %.5f mean %.5f" % (min(cs), sum(cs) / len(cs)))
    o, gx, gp = res["hip"]; a = res["autocast"]
    cs = [cos(p, q) for p, q in zip(gp, a[2])]
    print(ln, "hip vs autocast: fwd rel %.4f dx cos %.5f param cos min %.5f" % (((o - a[0]).norm() / a[0].norm()).item(), cos(gx, a[1]), min(cs)))
