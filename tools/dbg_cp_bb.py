"""Per-parameter accuracy of the dense backbone + neck alone: the CenterPoint backbone
(SECOND) + neck (SECONDFPN) of the tests/test_gpu_e2e_parity_centerpoint.py model, fed the float64 oracle's
sparse-encoder output E and its neck-output gradient dN, in float64 torch (CPU, the reference), fp32 torch on
the CPU and on the GPU (MIOpen), and the HIP fp32 engine. Prints every parameter gradient's relative L2 error
and the input gradient's, in module order."""
import copy
import sys

B = 2

import torch

sys.path.insert(0, ".")
from tests.test_gpu_e2e_parity_centerpoint import OracleStep, frames, init_mid_cell_offsets, oracle_voxels  # noqa: E402
from robustpointclouds_amd.trainer import Trainer, make_nus_model  # noqa: E402

rel = lambda a, b: float((a.double().cpu() - b.double().cpu()).norm() / b.double().cpu().norm().clamp_min(1e-30))
dev = torch.device("cuda")
torch.manual_seed(21)
model = make_nus_model(device=dev, epoch=3)
init_mid_cell_offsets(model)
Trainer._select_engines(model, bf16=False)
model.train()
pts, gts = frames()
rv, rc, rn = oracle_voxels(pts)
ogts = dict(boxes=[torch.from_numpy(b) for b, _ in gts], labels=[torch.from_numpy(l) for _, l in gts])

cap = {}


def hook(key):
    def h(mod, inp, out):
        lst = isinstance(out, (list, tuple))
        t = out[0] if lst else out
        cap[key] = t.detach().clone()
        if t.requires_grad:
            t.register_hook(lambda g: cap.__setitem__("d" + key, g.detach().clone()))
    return h


o = OracleStep(model, torch.float64)
o.ref.pts_middle_encoder.register_forward_hook(hook("E"))
o.ref.pts_neck.register_forward_hook(hook("N"))
o.step(rv, rn, rc, ogts)
E64, dN64 = cap["E"], cap["dN"]
print("E", tuple(E64.shape), "nonzero frac", float((E64 != 0).double().mean()), "dN", tuple(dN64.shape), flush=True)


def run(mode):
    bb, nk = copy.deepcopy(model.pts_backbone), copy.deepcopy(model.pts_neck)
    hip = mode == "hip32"
    for m in (bb, nk):
        if hasattr(m, "hip"):
            m.hip = hip
    if mode == "torch64":
        bb, nk, x, g = bb.cpu().double(), nk.cpu().double(), E64.clone(), dN64.clone()
    elif mode == "torch32cpu":
        bb, nk, x, g = bb.cpu().float(), nk.cpu().float(), E64.float(), dN64.float()
    else:
        bb, nk, x, g = bb.to(dev).float(), nk.to(dev).float(), E64.float().to(dev), dN64.float().to(dev)
        if hip:
            x = x.contiguous(memory_format=torch.channels_last)
    x.requires_grad_(True)
    out = nk(bb(x))[0]
    (out * g.to(out.dtype).view_as(out)).sum().backward()
    torch.cuda.synchronize()
    named = [("bb." + n, p.grad) for n, p in bb.named_parameters()] + [("nk." + n, p.grad) for n, p in nk.named_parameters()]
    return out.detach(), x.grad.detach(), named


ref = run("torch64")
res = {m: run(m) for m in ("torch32cpu", "torch32gpu", "hip32")}
print(f"{'':34s} " + " ".join(f"{m:>11s}" for m in res))
print(f"{'forward':34s} " + " ".join(f"{rel(r[0], ref[0]):11.2e}" for r in res.values()))
print(f"{'dE':34s} " + " ".join(f"{rel(r[1], ref[1]):11.2e}" for r in res.values()))
for i, (n, gr) in enumerate(ref[2]):
    print(f"{n:34s} " + " ".join(f"{rel(r[2][i][1], gr):11.2e}" for r in res.values()))
print("done")
