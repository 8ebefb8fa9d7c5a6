"""A/B of the sparse bf16 GEMM kernels (rpc_spconv_gemm_bf16_mode) inside the bf16 SparseEncoder forward +
backward on a synthetic KITTI batch (the metric's shapes): per mode, warm-up then timed steps (HIP events on
the stream). Run under `rocprofv3 --kernel-trace --stats` for per-kernel times of each mode.

    python tools/spgemm_ab.py [modes, default 0,1,2,3] [steps]"""
import sys
import time

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from robustpointclouds_amd import _ffi, voxelize  # noqa: E402
from robustpointclouds_amd.sparse_encoder import SparseEncoder  # noqa: E402
from robustpointclouds_amd.synthetic import KITTI_PC_RANGE, KITTI_VOXEL_SIZE, kitti_batch  # noqa: E402


def main():
    modes = [int(m) for m in (sys.argv[1] if len(sys.argv) > 1 else "0,1,2,3").split(",")]
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    lib = _ffi.load()
    dev = torch.device("cuda")
    pts, _, _ = kitti_batch(6, seed0=0, num_classes=3)
    pts = [torch.from_numpy(p).to(dev) for p in pts]
    d = voxelize.Voxelization(KITTI_VOXEL_SIZE, KITTI_PC_RANGE, 5, 16000).to(dev).voxelize_frames(pts)
    feats = (d["voxels"][:, :, :4].sum(1) / d["num_points"].clamp(min=1).view(-1, 1).float()).contiguous()
    coors = d["coors"]
    torch.manual_seed(0)
    enc = SparseEncoder(4, [41, 1600, 1408]).to(dev)
    enc.bf16 = enc.dense_nhwc = enc.dense_bf16 = True
    gout = None

    def step():
        nonlocal gout
        f = feats.clone().requires_grad_(True)
        out = enc(f, coors, 6)
        if gout is None:
            gout = torch.randn(out.shape, device=dev).to(out.dtype)
        out.backward(gout)

    for m in modes:
        lib.rpc_spconv_gemm_bf16_mode(m)
        for _ in range(5):
            step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        torch.cuda.synchronize()
        print(f"mode {m}: {1000 * (time.perf_counter() - t0) / steps:.3f} ms per encoder fwd+bwd", flush=True)


if __name__ == "__main__":
    main()
