"""Experiment: does a spatially coherent voxel row order speed up the sparse encoder? The same bench batches with
each frame's points sorted by the Morton code of their voxel (so the voxelizer's first-appearance order becomes a
Z-order of the voxels) against the generator's ring order, alternating A B A B in one process (same box, same
model), 3-class KITTI and CenterPoint. Prints ms/step per variant. (Sorting the points changes only which voxel
comes first; the voxel set, and so the work, is the same.)"""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
import bench  # noqa: E402
from robustpointclouds_amd.trainer import Trainer, make_kitti_model, make_nus_model  # noqa: E402


def morton_sort(p, vs, lo):
    q = np.floor((p[:, :3] - np.asarray(lo, np.float64)) / np.asarray(vs, np.float64)).astype(np.int64)
    q = np.clip(q, 0, (1 << 16) - 1)
    key = np.zeros(len(p), np.int64)
    for bit in range(16):
        for d in range(3):
            key |= ((q[:, d] >> bit) & 1) << (3 * bit + d)
    return p[np.argsort(key, kind="stable")]


def run(model_fn, data, steps, warm):
    torch.manual_seed(0)
    tr = Trainer(model_fn(), bf16=True, device=torch.device("cuda"))
    NB = len(data)
    ready = None
    for i in range(warm):
        tr.train_step(*data[i % NB], next_points=data[(i + 1) % NB][0])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        tr.train_step(*data[i % NB], next_points=data[(i + 1) % NB][0])
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps * 1e3


dev = torch.device("cuda")
ONLY = sys.argv[1] if len(sys.argv) > 1 else None   # "ring" / "morton": one kitti variant, 12 steps (for rocprofv3)
for name in (("kitti",) if ONLY else ("kitti", "nus")):
    if name == "kitti":
        data = bench._batches(4, 6, 0, dev, 3)
        vs, lo = (0.05, 0.05, 0.1), (0.0, -40.0, -3.0)
        mk = lambda: make_kitti_model(num_classes=3, device=dev, epoch=3)
        steps, warm = 30, 8
    else:
        data = bench._nus_batches(2, 4, 0, dev)
        vs, lo = (0.1, 0.1, 0.2), (-51.2, -51.2, -5.0)
        mk = lambda: make_nus_model(device=dev, epoch=3)
        steps, warm = 10, 4
    sdata = [([torch.from_numpy(morton_sort(p.cpu().numpy(), vs, lo)).to(dev) for p in pts], gt) for pts, gt in data]
    if ONLY:
        print(ONLY, run(mk, data if ONLY == "ring" else sdata, 8, 4), flush=True)
        break
    res = {"ring": [], "morton": []}
    for rep in range(2):
        res["ring"].append(run(mk, data, steps, warm))
        res["morton"].append(run(mk, sdata, steps, warm))
        print(name, rep, {k: round(v[-1], 3) for k, v in res.items()}, flush=True)
    print(name, "ms/step ring", [round(v, 3) for v in res["ring"]], "morton", [round(v, 3) for v in res["morton"]],
          flush=True)
