"""Training-stream idle time between bench steps, without a profiler: a timing event is recorded on the training
stream when Trainer.train_step is entered (before any of the step's kernels is issued) and when it returns; the
GPU time from one step's end event to the next step's start event is time the stream sat idle waiting for the
host to issue work (0 when the host ran ahead). Also the GPU span of each step.

    python tools/step_gaps.py [--steps 30]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from robustpointclouds_amd.trainer import Trainer, make_kitti_model  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=30)
    a = ap.parse_args()
    dev = torch.device("cuda")
    torch.manual_seed(0)
    model = make_kitti_model(num_classes=3, device=dev, epoch=3)
    tr = Trainer(model, bf16=True, device=dev)
    data = bench._batches(4, 6, 0, dev, 3)
    ready = torch.cuda.Event()
    ready.record()
    for i in range(8):
        tr.train_step(*data[i % 4], next_points=data[(i + 1) % 4][0], next_ready=ready)
    torch.cuda.synchronize()
    ev = []
    for i in range(a.steps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        tr.train_step(*data[i % 4], next_points=data[(i + 1) % 4][0], next_ready=ready)
        e1.record()
        ev.append((e0, e1))
    torch.cuda.synchronize()
    spans = [a_.elapsed_time(b_) for a_, b_ in ev]
    gaps = [ev[i][1].elapsed_time(ev[i + 1][0]) for i in range(len(ev) - 1)]
    tot = ev[0][0].elapsed_time(ev[-1][1])
    print(f"{a.steps} steps: {tot / a.steps:.3f} ms/step; step span median {sorted(spans)[len(spans) // 2]:.3f} ms; "
          f"inter-step idle median {sorted(gaps)[len(gaps) // 2]:.3f} ms, mean {sum(gaps) / len(gaps):.3f} ms")


if __name__ == "__main__":
    main()
