"""Where the small copy / fill launches of a training step come from: torch.profiler over eager steps of the
bench workload (RPC_DENSE_GRAPHS=0, so every launch has a host-side caller), the device kernels of each op
grouped by kernel name and the innermost package frame of the op's Python stack, per step.

    RPC_DENSE_GRAPHS=0 python tools/step_copies.py [--steps 2] [--classes 3]
"""
import argparse
import collections
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import bench  # noqa: E402

KEYS = ("Memcpy", "Memset", "copyBuffer", "fillBuffer", "FillFunctor", "elementwise", "CatArray", "rocprim", "reduce", "copy_kernel")


def _site(evt):
    for fr in evt.stack or ():
        if "robustpointclouds_amd" in fr or "bench.py" in fr:
            return fr.split("robustpointclouds_amd/")[-1]
    return (evt.stack or ["?"])[0]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--classes", type=int, default=3)
    a = ap.parse_args()
    from robustpointclouds_amd.trainer import Trainer, make_kitti_model
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = make_kitti_model(num_classes=a.classes, device=dev, epoch=3)
    tr = Trainer(model, bf16=True, device=dev)
    data = bench._batches(2, 6, 0, dev, a.classes)
    for i in range(4):
        tr.train_step(*data[i % 2])
    torch.cuda.synchronize()
    acts = [torch.profiler.ProfilerActivity.CPU, torch.profiler.ProfilerActivity.CUDA]
    with torch.profiler.profile(activities=acts, with_stack=True, acc_events=True, record_shapes=True) as prof:
        for i in range(a.steps):
            tr.train_step(*data[i % 2])
        torch.cuda.synchronize()
    by = collections.Counter()
    dur = collections.Counter()
    total = collections.Counter()
    for evt in prof.events():
        for k in getattr(evt, "kernels", ()) or ():
            total[k.name] += 1
            if any(s in k.name for s in KEYS):
                key = (k.name[:60], evt.name, _site(evt) if "Memcpy" not in k.name else
                       f"{evt.input_shapes} thread {evt.thread}")
                by[key] += 1
                dur[key] += k.duration
    print(f"{a.steps} eager steps; copy / fill / small-op kernels by (kernel, op, innermost package frame), per step:")
    for key, n in by.most_common():
        print(f"  {n / a.steps:5.1f}  {dur[key] / n:7.1f} us  {key[0]:60s} {key[1]:28s} {key[2]}")
    print("runtime copies / fills without an op (hipMemcpyAsync / hipMemsetAsync from the library):")
    kt = collections.Counter()
    for evt in prof.events():
        if any(s in evt.name for s in ("copyBuffer", "fillBuffer", "Memcpy", "Memset")):
            kt[(evt.name[:60], str(evt.device_type))] += 1
    for k, n in kt.most_common():
        print(f"  {n / a.steps:5.1f}  {k}  (all launches, with or without an op)")
    # Python call sites of the aten copies / fills on CUDA tensors (a TorchDispatchMode over one step, the backward
    # on this thread so its Python frames are seen too)
    import traceback
    from torch.utils._python_dispatch import TorchDispatchMode
    sites = collections.Counter()

    class Mode(TorchDispatchMode):
        def __torch_dispatch__(self, func, types, args=(), kwargs=None):
            nm = str(func)
            if any(k in nm for k in ("copy", "fill", "zero", "cat", "clone")):
                fr = [f for f in traceback.extract_stack()[:-1] if "robustpointclouds_amd" in f.filename
                      or f.filename.endswith("bench.py")]
                where = " < ".join(f"{f.filename.split('/')[-1]}:{f.lineno}" for f in fr[::-1][:3]) if fr else "?"
                sites[(nm, where)] += 1
            return func(*args, **(kwargs or {}))

    torch.autograd.set_multithreading_enabled(False)
    with Mode():
        tr.train_step(*data[0])
    torch.cuda.synchronize()
    print("aten copy / fill / cat call sites in one step (op, innermost package frames):")
    for (nm, where), n in sorted(sites.items(), key=lambda kv: -kv[1]):
        print(f"  {n:4d}  {nm:28s} {where}")


if __name__ == "__main__":
    main()
