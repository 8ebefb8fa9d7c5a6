"""Debug the CenterPoint fp32 e2e gradient gap: loss-gradient and head-input-gradient of the HIP step vs the
float64 oracle composition (same setup as tests/test_gpu_e2e_parity_centerpoint.py)."""
import sys

B = 2   # the r04 case: frames() defaults (2 one-sweep frames)

import torch

sys.path.insert(0, ".")
from tests.test_gpu_e2e_parity_centerpoint import OracleStep, frames, oracle_voxels  # noqa: E402
from robustpointclouds_amd.adversarial_loss import parse_losses  # noqa: E402
from robustpointclouds_amd.center_head import pack_gt  # noqa: E402
from robustpointclouds_amd.trainer import Trainer, make_nus_model  # noqa: E402

rel = lambda a, b: float((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30))
dev = torch.device("cuda")
torch.manual_seed(21)
model = make_nus_model(device=dev, epoch=3)
with torch.no_grad():
    for th in model.pts_bbox_head.task_heads:
        for dcn in (th.feature_adapt_cls, th.feature_adapt_reg):
            dcn.conv_offset.weight.normal_(0, 0.02)
            dcn.conv_offset.bias.uniform_(-0.5, 0.5)
Trainer._select_engines(model, bf16=False)
model.train()
pts, gts = frames()
o64 = OracleStep(model, torch.float64)
cap = {}


def keep(name):
    def hook(mod, inp, out):
        t = out[0] if isinstance(out, (list, tuple)) else out
        cap[name] = t
        if t.requires_grad:
            t.register_hook(lambda g: cap.__setitem__(name + ".grad", g))
    return hook


model.pts_neck.register_forward_hook(keep("neck"))
model.pts_backbone.register_forward_hook(keep("backbone"))
o64.ref.pts_neck.register_forward_hook(keep("o.neck"))
o64.ref.pts_backbone.register_forward_hook(keep("o.backbone"))
gpts = [torch.from_numpy(p).to(dev) for p in pts]
batch = model.data_preprocessor(dict(inputs=dict(points=gpts)), training=True)["inputs"]
batch["batch_size"] = B
gb, gl = pack_gt([torch.from_numpy(b) for b, _ in gts], [torch.from_numpy(l) for _, l in gts], dev)
losses = model.loss(batch, dict(gt_boxes=gb, gt_labels=gl))
total, _ = parse_losses(losses)
total.backward()
torch.cuda.synchronize()
rv, rc, rn = oracle_voxels(pts)
ogts = dict(boxes=[torch.from_numpy(b) for b, _ in gts], labels=[torch.from_numpy(l) for _, l in gts])
o64.step(rv, rn, rc, ogts)
for k in ("backbone", "neck"):
    a, b = cap[k], cap["o." + k]
    a = a[0] if isinstance(a, (list, tuple)) else a
    b = b[0] if isinstance(b, (list, tuple)) else b
    print(k, "fwd rel", rel(a.detach().float().cpu(), b.detach()), "grad rel",
          rel(cap[k + ".grad"].float().cpu(), cap["o." + k + ".grad"]) if k + ".grad" in cap and "o." + k + ".grad" in cap else None)
