"""Where do the step's small torch kernels / copies / fills come from? torch.profiler over one bench step of the
metric's model (3-class, B=6, bf16 perf mode) with Python stacks; prints every aten op that ran device work,
grouped by its innermost robustpointclouds_amd call site."""
import collections
import sys

import torch
from torch.profiler import ProfilerActivity, profile

sys.path.insert(0, ".")
from robustpointclouds_amd.anchor_head import pack_gt  # noqa: E402
from robustpointclouds_amd.synthetic import kitti_batch  # noqa: E402
from robustpointclouds_amd.trainer import Trainer, make_kitti_model  # noqa: E402

dev = torch.device("cuda")
torch.manual_seed(0)
if len(sys.argv) > 1 and sys.argv[1] == "centerpoint":
    import bench
    from robustpointclouds_amd.trainer import make_nus_model
    model = make_nus_model(device=dev, epoch=3)
    gpts, gt = bench._nus_batches(1, 4, 0, dev)[0]
else:
    model = make_kitti_model(num_classes=3, device=dev, epoch=3)
    pts, boxes, labels = kitti_batch(6, seed0=0, num_classes=3)
    gpts = [torch.from_numpy(p).to(dev) for p in pts]
    gb, gl = pack_gt(list(zip(boxes, labels)), dev)
    gt = dict(gt_boxes=gb, gt_labels=gl)
tr = Trainer(model, bf16=True, device=dev)
for _ in range(4):
    tr.train_step(gpts, gt, next_points=gpts)
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True,
             experimental_config=torch._C._profiler._ExperimentalConfig(verbose=True)) as prof:
    tr.train_step(gpts, gt, next_points=gpts)
    torch.cuda.synchronize()
sites = collections.Counter()
dev_us = collections.Counter()
for ev in prof.events():
    if not ev.name.startswith("aten::") and "Memcpy" not in ev.name and "Memset" not in ev.name:
        continue
    t = ev.device_time_total if hasattr(ev, "device_time_total") else ev.cuda_time_total
    if t <= 0 or ev.cpu_parent is not None and ev.cpu_parent.name.startswith("aten::"):
        continue
    stack = [s for s in (ev.stack or []) if "torch/" not in s and "<built-in" not in s]
    site = " <- ".join(x.split("/")[-1] for x in stack[:3]) if stack else "?"
    key = f"{ev.name:28s} {site}"
    sites[key] += 1
    dev_us[key] += t
for k, n in sorted(sites.items(), key=lambda kv: -dev_us[kv[0]]):
    print(f"{n:3d} x {dev_us[k] / n:7.1f} us  {k}")
