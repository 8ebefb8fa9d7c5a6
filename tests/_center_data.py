"""Synthetic nuScenes-like GT boxes for the CenterHead tests (seeded numpy)."""
import numpy as np
import torch


def nus_gts(B, seed, n=30, ncls=10, edge_cases=True):
    """Per frame [n, 9] LiDAR boxes (bottom centre) and [n] labels inside/around the 102.4 m BEV."""
    rng = np.random.default_rng(seed)
    out = []
    for b in range(B):
        k = int(n + rng.integers(-5, 6))
        xy = rng.uniform(-54.0, 54.0, (k, 2))           # a few outside the range
        z = rng.uniform(-3.0, 1.0, (k, 1))
        dims = np.stack([rng.uniform(0.4, 3.0, k), rng.uniform(0.4, 12.0, k), rng.uniform(0.8, 4.0, k)], 1)
        rot = rng.uniform(-np.pi, np.pi, (k, 1))
        vel = rng.normal(0, 3.0, (k, 2))
        boxes = np.concatenate([xy, z, dims, rot, vel], 1).astype(np.float32)
        labels = rng.integers(0, ncls, k).astype(np.int64)
        if edge_cases and k > 6:
            boxes[1, 3] = 0.0                            # zero width: skipped
            boxes[3, :2] = boxes[2, :2] + 0.01           # same centre cell as box 2
            labels[3] = labels[2]
            boxes[4, :2] = (51.19, -51.2)                # last / first cell
            labels[5] = 99                               # out-of-range label: ignored
        out.append((torch.from_numpy(boxes), torch.from_numpy(labels)))
    return out
