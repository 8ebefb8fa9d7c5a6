"""Perturber timing alone (the metric's VoxelPerturber, 3-class SECOND config): fused perturb_voxels forward +
backward on synthetic voxels (V voxels x 5 slots x 4 features, 1..5 valid slots each), HIP-event ms per call at
several voxel counts — time(N) = fixed + per-point, which says how much of the ~0.85 ms per step is per-point
work (MFMA, bytes) and how much is launch / hand-off latency. Run under rocprofv3 --kernel-trace --stats for
the per-kernel split.

    python tools/pert_bench.py [V1,V2,...]   (default 10000,20000,40000,80000; ~2.8 valid points per voxel)
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from robustpointclouds_amd.trainer import make_kitti_model  # noqa: E402


def voxels_of(V, dev, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    npts = torch.randint(1, 6, (V,), generator=g)
    vox = torch.zeros(V, 5, 4)
    slot = torch.arange(5).view(1, 5)
    mask = slot < npts.view(-1, 1)
    vals = torch.rand(V, 5, 4, generator=g) * torch.tensor([70.0, 80.0, 4.0, 1.0]) + torch.tensor([0.0, -40.0, -3.0, 0.01])
    vox[mask] = vals[mask]
    return vox.to(dev), npts.to(torch.int32).to(dev), int(mask.sum())


def main():
    Vs = [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "10000,20000,40000,80000").split(",")]
    dev = torch.device("cuda")
    torch.manual_seed(0)
    model = make_kitti_model(num_classes=3, device=dev, epoch=3)
    model.train()
    adv = model.adversary
    adv.wgrad_split_bf16 = True    # as the bench's bf16 Trainer sets it (base_model.py)
    for V in Vs:
        vox, npts, nvalid = voxels_of(V, dev)

        def fwd():
            vfe, ld, _, _ = adv.perturb_voxels(vox, npts, 4)
            return vfe, ld

        def fwd_bwd():
            vfe, ld = fwd()
            (vfe.sum() + sum(v for v in ld.values() if torch.is_tensor(v) and v.requires_grad)).backward()

        res = {}
        for name, fn in (("fwd", fwd), ("fwd+bwd", fwd_bwd)):
            for _ in range(3):
                fn()
            torch.cuda.synchronize()
            ts = []
            for _ in range(5):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(10):
                    fn()
                e1.record()
                e1.synchronize()
                ts.append(e0.elapsed_time(e1) / 10)
            res[name] = sorted(ts)[2]
        print(f"V {V:6d} valid points {nvalid:7d}  fwd {res['fwd']:.3f} ms  fwd+bwd {res['fwd+bwd']:.3f} ms", flush=True)


if __name__ == "__main__":
    main()
