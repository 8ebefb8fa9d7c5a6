"""Host-side (Python) time per training step: cProfile over K steps of the bench workload.

    python tools/host_profile.py [--steps 20] [--classes 1]
"""
import argparse
import cProfile
import os
import pstats
import sys

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
    data = bench._batches(2, 6, 0, dev, a.classes)
    for i in range(5):
        tr.train_step(*data[i % 2])
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    pr.enable()
    for i in range(a.steps):
        tr.train_step(*data[i % 2])
    torch.cuda.synchronize()
    pr.disable()
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(45)
    st.sort_stats("cumulative").print_stats(60)


if __name__ == "__main__":
    main()
