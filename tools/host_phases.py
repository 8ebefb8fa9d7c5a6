"""Host time per phase of the bench step (no GPU sync added): how long the Python host spends issuing
each autograd node's kernels, and how long it waits in host reads / event waits.

    python tools/host_phases.py [--steps 20] [--classes 3]

Each phase is timed with time.perf_counter around the node's forward / backward (the autograd engine
runs backward nodes on its own thread, so backward phases are timed there). Blocking waits are timed
separately (torch.cuda.Event.synchronize, Tensor.item). GPU time per step is printed for comparison:
where a phase's host time exceeds the GPU time of the kernels it issues, the GPU waits on the host.
"""
import argparse
import collections
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import bench  # noqa: E402

T = collections.defaultdict(float)
N = collections.defaultdict(int)


def wrap_static(cls, name, tag):
    f = getattr(cls, name)

    def g(*a, **k):
        t0 = time.perf_counter()
        try:
            return f(*a, **k)
        finally:
            T[tag] += time.perf_counter() - t0
            N[tag] += 1
    setattr(cls, name, staticmethod(g))


def wrap_method(cls, name, tag):
    f = getattr(cls, name)

    def g(self, *a, **k):
        t0 = time.perf_counter()
        try:
            return f(self, *a, **k)
        finally:
            T[tag] += time.perf_counter() - t0
            N[tag] += 1
    setattr(cls, name, g)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--classes", type=int, default=3)
    a = ap.parse_args()
    from robustpointclouds_amd import anchor_head, dense_bev, optim, perturb, sparse_encoder, trainer, voxelize
    from robustpointclouds_amd.adversarial_loss import LossTailFn
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = trainer.make_kitti_model(num_classes=a.classes, device=dev, epoch=3)
    tr = trainer.Trainer(model, bf16=True, device=dev)
    data = bench._batches(4, 6, 0, dev, a.classes)
    ready = torch.cuda.Event()
    ready.record()
    for i in range(8):
        tr.train_step(*data[i % 4], next_points=data[(i + 1) % 4][0], next_ready=ready)
    torch.cuda.synchronize()
    for cls, tag in ((perturb.PerturbVoxelsFn, "perturber"), (sparse_encoder.SparseEncoderFn, "sparse"),
                     (dense_bev.BackboneFn, "second"), (dense_bev.NeckFn, "fpn"), (anchor_head.HeadLossFn, "head_loss"),
                     (LossTailFn, "loss_tail")):
        wrap_static(cls, "forward", tag + ".fwd")
        wrap_static(cls, "backward", tag + ".bwd")
    wrap_method(optim.ClipAdamW, "step", "optimizer")
    wrap_method(trainer.Trainer, "_prefetch", "prefetch_voxelize")
    wrap_method(voxelize.PendingVoxels, "result", "wait_V")
    wrap_method(torch.cuda.Event, "synchronize", "event_sync (blocking)")
    wrap_method(torch.Tensor, "item", "item (blocking)")
    wrap_method(trainer.Trainer, "train_step", "train_step total")
    T.clear()
    N.clear()
    t0 = time.perf_counter()
    for i in range(a.steps):
        tr.train_step(*data[i % 4], next_points=data[(i + 1) % 4][0], next_ready=ready)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    n = a.steps
    print(f"wall/step {1e3 * (t2 - t0) / n:.3f} ms, host issue/step {1e3 * (t1 - t0) / n:.3f} ms, "
          f"drain {1e3 * (t2 - t1):.3f} ms")
    for k in sorted(T, key=lambda k: -T[k]):
        print(f"  {k:28s} {1e3 * T[k] / n:8.3f} ms/step  ({N[k] / n:.1f} calls/step)")


if __name__ == "__main__":
    main()
