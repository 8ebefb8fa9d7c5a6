"""Host-bound check of the bench step: time blocked inside each host read (Tensor.item) vs host busy time.

    python tools/host_gap.py [--steps 20] [--classes 1]
If host busy time per step approaches the GPU time per step, the step is host-issue bound.
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--classes", type=int, default=1)
    a = ap.parse_args()
    from robustpointclouds_amd.trainer import Trainer, make_kitti_model
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = make_kitti_model(num_classes=a.classes, device=dev, epoch=3)
    tr = Trainer(model, bf16=True, device=dev)
    data = bench._batches(4, 6, 0, dev, a.classes)
    for i in range(8):
        tr.train_step(*data[i % 4])
    torch.cuda.synchronize()
    orig = torch.Tensor.item
    log = []

    def item(self):
        t0 = time.perf_counter()
        v = orig(self)
        log.append((t0, time.perf_counter()))
        return v
    torch.Tensor.item = item
    steps = []
    t_start = time.perf_counter()
    for i in range(a.steps):
        t0 = time.perf_counter()
        tr.train_step(*data[i % 4])
        steps.append((t0, time.perf_counter()))
    t_issue = time.perf_counter()
    torch.cuda.synchronize()
    t_end = time.perf_counter()
    torch.Tensor.item = orig
    blocked = sum(b - a for a, b in log)
    wall = t_end - t_start
    n = a.steps
    print(f"steps {n}: wall/step {1e3 * wall / n:.3f} ms, host call/step {1e3 * (t_issue - t_start) / n:.3f} ms, "
          f"blocked in {len(log) / n:.1f} item()/step {1e3 * blocked / n:.3f} ms/step, host busy/step "
          f"{1e3 * (t_issue - t_start - blocked) / n:.3f} ms, drain after last issue {1e3 * (t_end - t_issue):.3f} ms")
    # per-read blocked time of the last step
    s0, s1 = steps[-1]
    per = [(round(1e3 * (x - s0), 3), round(1e6 * (y - x), 1)) for x, y in log if s0 <= x <= s1]
    print("last step: (ms into step, us blocked) per host read:", per)


if __name__ == "__main__":
    main()
