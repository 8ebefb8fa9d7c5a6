"""Same-process A/B of the fused AdversarialCenterPoint loss tail (rpc_center_tail_*) against the torch composition
it replaces (fused_center_tail patched to decline), on the config-4 bench batches: A B A B, ms/step."""
import sys
import time

import torch

sys.path.insert(0, ".")
import bench  # noqa: E402
import robustpointclouds_amd.plugin.models.detectors.adversarial_centerpoint as acp  # noqa: E402
from robustpointclouds_amd.trainer import Trainer, make_nus_model  # noqa: E402

dev = torch.device("cuda")
data = bench._nus_batches(2, 4, 0, dev)
orig = acp.fused_center_tail


def run(fused, steps=10, warm=4):
    acp.fused_center_tail = orig if fused else (lambda *a, **k: None)
    torch.manual_seed(0)
    tr = Trainer(make_nus_model(device=dev, epoch=3), bf16=True, device=dev)
    for i in range(warm):
        tr.train_step(*data[i % 2], next_points=data[(i + 1) % 2][0])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        tr.train_step(*data[i % 2], next_points=data[(i + 1) % 2][0])
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps * 1e3


res = {"fused": [], "torch": []}
for rep in range(2):
    res["fused"].append(run(True))
    res["torch"].append(run(False))
    print(rep, {k: round(v[-1], 3) for k, v in res.items()}, flush=True)
print("ms/step fused", [round(v, 3) for v in res["fused"]], "torch", [round(v, 3) for v in res["torch"]], flush=True)
