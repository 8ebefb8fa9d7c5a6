"""cProfile of the bench step's host side (N steps after warm-up): which Python functions the host
spends its issue time in.   python tools/host_cprofile.py [--steps 10]"""
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
    ap.add_argument("--steps", type=int, default=10)
    a = ap.parse_args()
    from robustpointclouds_amd import trainer
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = trainer.make_kitti_model(num_classes=3, device=dev, epoch=3)
    tr = trainer.Trainer(model, bf16=True, device=dev)
    data = bench._batches(4, 6, 0, dev, 3)
    ready = torch.cuda.Event()
    ready.record()
    for i in range(8):
        tr.train_step(*data[i % 4], next_points=data[(i + 1) % 4][0], next_ready=ready)
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    pr.enable()
    for i in range(a.steps):
        tr.train_step(*data[i % 4], next_points=data[(i + 1) % 4][0], next_ready=ready)
    pr.disable()
    torch.cuda.synchronize()
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(45)
    st.sort_stats("cumulative").print_stats(45)


if __name__ == "__main__":
    main()
