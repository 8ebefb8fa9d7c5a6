"""Host-bound check of the bench step: time blocked inside each host read (Tensor.item) vs host busy time.

    python tools/host_gap.py [--steps 20] [--classes 1] [--model voxelnet|centerpoint]
If host busy time per step approaches the GPU time per step, the step is host-issue bound. Host reads are
Tensor.item and Event.synchronize (the voxelizer's and sparse encoder's shape reads).
"""
import argparse
import os
import sys
import time
import traceback

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--classes", type=int, default=1)
    ap.add_argument("--model", default="voxelnet")
    a = ap.parse_args()
    from robustpointclouds_amd.trainer import Trainer, make_kitti_model, make_nus_model
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    if a.model == "centerpoint":
        model = make_nus_model(device=dev, epoch=3)
        data = bench._nus_batches(4, 4, 0, dev)
    else:
        model = make_kitti_model(num_classes=a.classes, device=dev, epoch=3)
        data = bench._batches(4, 6, 0, dev, a.classes)
    tr = Trainer(model, bf16=True, device=dev)
    NB = len(data)
    ready = torch.cuda.Event()    # as bench.py: the synthetic frames are resident once, nothing to wait for
    ready.record(torch.cuda.current_stream(dev))
    for i in range(8):
        tr.train_step(*data[i % NB], next_points=data[(i + 1) % NB][0], next_ready=ready)
    torch.cuda.synchronize()
    orig, orig_ev = torch.Tensor.item, torch.cuda.Event.synchronize
    log = []

    def timed(fn):
        def w(self):
            t0 = time.perf_counter()
            v = fn(self)
            site = [f"{os.path.basename(f.filename)}:{f.lineno}" for f in traceback.extract_stack()[:-1]
                    if "robustpointclouds_amd" in f.filename or "trainer" in f.filename]
            log.append((t0, time.perf_counter(), " <- ".join(reversed(site[-3:]))))
            return v
        return w
    torch.Tensor.item = timed(orig)
    torch.cuda.Event.synchronize = timed(orig_ev)
    steps = []
    t_start = time.perf_counter()
    for i in range(a.steps):
        t0 = time.perf_counter()
        tr.train_step(*data[i % NB], next_points=data[(i + 1) % NB][0], next_ready=ready)
        steps.append((t0, time.perf_counter()))
    t_issue = time.perf_counter()
    torch.cuda.synchronize()
    t_end = time.perf_counter()
    torch.Tensor.item, torch.cuda.Event.synchronize = orig, orig_ev
    blocked = sum(b - a for a, b, _ in log)
    wall = t_end - t_start
    n = a.steps
    print(f"steps {n}: wall/step {1e3 * wall / n:.3f} ms, host call/step {1e3 * (t_issue - t_start) / n:.3f} ms, "
          f"blocked in {len(log) / n:.1f} host reads/step {1e3 * blocked / n:.3f} ms/step, host busy/step "
          f"{1e3 * (t_issue - t_start - blocked) / n:.3f} ms, drain after last issue {1e3 * (t_end - t_issue):.3f} ms")
    # per-read blocked time of the last step
    s0, s1 = steps[-1]
    print("last step: ms into step, us blocked, call site per host read:")
    for x, y, site in log:
        if s0 <= x <= s1:
            print(f"  {1e3 * (x - s0):8.3f} {1e6 * (y - x):9.1f}  {site}")


if __name__ == "__main__":
    main()
