"""Localise the CenterPoint fp32 gradient gap by substitution: run the HIP step and the
float64 / fp32 oracle compositions of tests/test_gpu_e2e_parity_centerpoint.py with the sparse-encoder output
(E) or the neck output (N) of one side fed into the other side's downstream (value substitution, the gradient
still flows through the receiving side's own upstream), and report each run's gradients against plain float64."""
import sys

B = 2   # the r04 case: frames() defaults (2 one-sweep frames)
import time

import torch

sys.path.insert(0, ".")
from tests.test_gpu_e2e_parity_centerpoint import (OracleStep, frames, hip_grads, init_mid_cell_offsets,  # noqa: E402
                                                   oracle_voxels)
from robustpointclouds_amd.adversarial_loss import parse_losses  # noqa: E402
from robustpointclouds_amd.center_head import pack_gt  # noqa: E402
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
gpts = [torch.from_numpy(p).to(dev) for p in pts]
gb, gl = pack_gt([torch.from_numpy(b) for b, _ in gts], [torch.from_numpy(l) for _, l in gts], dev)


def subst_hook(cap, key, sub=None):
    """forward hook: record the module output (and its gradient); with `sub`, replace its value."""
    def hook(mod, inp, out):
        lst = isinstance(out, (list, tuple))
        t = out[0] if lst else out
        if sub is not None:
            s = t.detach().clone()
            s.copy_(sub.to(device=t.device, dtype=t.dtype).view_as(t))
            t = t + (s - t).detach()
        cap[key] = t.detach().clone()
        if t.requires_grad:
            t.register_hook(lambda g: cap.__setitem__("d" + key, g.detach().clone()))
        return [t] if lst else t
    return hook


def hip_run(subE=None, subN=None):
    model.zero_grad(set_to_none=True)
    cap = {}
    hs = [model.pts_middle_encoder.register_forward_hook(subst_hook(cap, "E", subE)),
          model.pts_neck.register_forward_hook(subst_hook(cap, "N", subN))]
    batch = model.data_preprocessor(dict(inputs=dict(points=gpts)), training=True)["inputs"]
    batch["batch_size"] = B
    losses = model.loss(batch, dict(gt_boxes=gb, gt_labels=gl))
    total, _ = parse_losses(losses)
    total.backward()
    torch.cuda.synchronize()
    for h in hs:
        h.remove()
    g = [(n, t.detach().cpu().clone()) for n, t in hip_grads(model)]
    return g, cap, float(total)


def oracle_run(dtype, subE=None, subN=None):
    t0 = time.time()
    o = OracleStep(model, dtype)
    cap = {}
    o.ref.pts_middle_encoder.register_forward_hook(subst_hook(cap, "E", subE))
    o.ref.pts_neck.register_forward_hook(subst_hook(cap, "N", subN))
    o.step(rv, rn, rc, ogts)
    g = [(n, t.detach().clone()) for n, t in o.grads()]
    print(f"  (oracle {dtype} {time.time() - t0:.1f} s)", flush=True)
    return g, cap, float(o.total)


GROUPS = ("adversary", "middle", "backbone", "neck", "head")
WATCH = ("adversary.Wa1", "adversary.W5", "middle.0.W", "backbone.blocks.0.1.weight",
         "head.task_heads.3.feature_adapt_cls.conv_offset.weight", "head.shared_conv.conv.weight")


def report(tag, g, ref):
    rows = {n: rel(a, r) for (n, a), (_, r) in zip(g, ref)}
    s = f"{tag:34s} mean {sum(rows.values()) / len(rows):.2e} max {max(rows.values()):.2e} |"
    for grp in GROUPS:
        v = [e for n, e in rows.items() if n.startswith(grp)]
        s += f" {grp} {max(v):.1e}/{sum(v) / len(v):.1e}"
    print(s)
    print("      " + " ".join(f"{w.split('.')[-2] if 'head' in w else w}={rows[w]:.1e}" for w in WATCH))
    return rows


print("HIP plain", flush=True)
g_hip, c_hip, t_hip = hip_run()
print("oracle f64 plain", flush=True)
g64, c64, t64 = oracle_run(torch.float64)
print("oracle f32 plain", flush=True)
g32, c32, t32 = oracle_run(torch.float32)
print(f"forward: E hip {rel(c_hip['E'], c64['E']):.2e} f32 {rel(c32['E'], c64['E']):.2e}; "
      f"N hip {rel(c_hip['N'], c64['N']):.2e} f32 {rel(c32['N'], c64['N']):.2e}; "
      f"dN hip {rel(c_hip['dN'], c64['dN']):.2e} f32 {rel(c32['dN'], c64['dN']):.2e}; "
      f"dE hip {rel(c_hip['dE'], c64['dE']):.2e} f32 {rel(c32['dE'], c64['dE']):.2e}; "
      f"total hip {t_hip} f32 {t32} f64 {t64}", flush=True)

report("HIP", g_hip, g64)
report("oracle f32", g32, g64)

print("HIP with E := E64", flush=True)
g, c, _ = hip_run(subE=c64["E"])
report("HIP | E64", g, g64)
print(f"   N {rel(c['N'], c64['N']):.2e} dN {rel(c['dN'], c64['dN']):.2e} dE {rel(c['dE'], c64['dE']):.2e}")

print("HIP with N := N64", flush=True)
g, c, _ = hip_run(subN=c64["N"])
report("HIP | N64", g, g64)
print(f"   dN {rel(c['dN'], c64['dN']):.2e} dE {rel(c['dE'], c64['dE']):.2e}")

print("oracle f64 with E := E_hip", flush=True)
g, c, _ = oracle_run(torch.float64, subE=c_hip["E"])
report("f64 | E_hip", g, g64)
print(f"   N {rel(c['N'], c64['N']):.2e} dN {rel(c['dN'], c64['dN']):.2e} dE {rel(c['dE'], c64['dE']):.2e}")

print("oracle f64 with E := E32", flush=True)
g, c, _ = oracle_run(torch.float64, subE=c32["E"])
report("f64 | E32", g, g64)

print("oracle f64 with N := N_hip", flush=True)
g, c, _ = oracle_run(torch.float64, subN=c_hip["N"])
report("f64 | N_hip", g, g64)
print(f"   dN {rel(c['dN'], c64['dN']):.2e} dE {rel(c['dE'], c64['dE']):.2e}")

print("oracle f64 with N := N32", flush=True)
g, c, _ = oracle_run(torch.float64, subN=c32["N"])
report("f64 | N32", g, g64)
print("done")
