"""Timing attribution of the sparse bf16 GEMM k_gemm_bf16<64, 4, ·> (rpc_spconv_gemm_bf16_mode 4 + DBG arms:
1 no MFMA, 2 gathers out of range, 4 weight loads out of range, 8 no gather instructions) on the real
64 x 64 rulebooks of a synthetic KITTI batch: HIP-event time per launch of each arm.
    python tools/spgemm_arms.py"""
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from robustpointclouds_amd import _ffi, voxelize  # noqa: E402
from robustpointclouds_amd.sparse_encoder import SparseEncoder  # noqa: E402
from robustpointclouds_amd.synthetic import KITTI_PC_RANGE, KITTI_VOXEL_SIZE, kitti_batch  # noqa: E402


def main():
    lib = _ffi.load()
    dev = torch.device("cuda")
    pts, _, _ = kitti_batch(6, seed0=0, num_classes=3)
    pts = [torch.from_numpy(p).to(dev) for p in pts]
    d = voxelize.Voxelization(KITTI_VOXEL_SIZE, KITTI_PC_RANGE, 5, 16000).to(dev).voxelize_frames(pts)
    feats = (d["voxels"][:, :, :4].sum(1) / d["num_points"].clamp(min=1).view(-1, 1).float()).contiguous()
    enc = SparseEncoder(4, [41, 1600, 1408]).to(dev)
    enc.bf16 = enc.dense_nhwc = enc.dense_bf16 = True
    enc.flop_probe = []
    enc(feats, d["coors"], 6)
    torch.cuda.synchronize()
    # the 64 -> 64 submanifold layers' rulebooks (subm3, subm4)
    cases = [(nbr, ci, co) for nbr, ci, co in enc.flop_probe[-1] if ci == 64 and co == 64 and nbr.shape[1] == 27]
    seen = set()
    for nbr, ci, co in cases:
        if nbr.data_ptr() in seen:
            continue
        seen.add(nbr.data_ptr())
        n = nbr.shape[0]
        a = torch.randn((n, 64), device=dev).to(torch.bfloat16)
        W = torch.randn((27, 64, 64), device=dev) * 0.05
        bt = torch.empty(lib.rpc_spconv_bf16_weight_elems(27, 64, 64, 0), dtype=torch.bfloat16, device=dev)
        _ffi.check(lib.rpc_spconv_prep_weight_bf16(_ffi.ptr(W), 27, 64, 64, 0, _ffi.ptr(bt), _ffi.stream_of(W)), "prep")
        out = torch.empty((n, 64), device=dev)
        part = torch.empty((lib.rpc_spconv_gemm_blocks(n), 128), device=dev)
        pairs = int((nbr >= 0).sum().item())
        for mode in [0, 4, 5, 6, 7, 8, 9, 12, 13, 1]:
            lib.rpc_spconv_gemm_bf16_mode(mode)
            ts = []
            for it in range(30):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                _ffi.check(lib.rpc_spconv_gemm_bf16_n(_ffi.ptr(a), n, 64, _ffi.ptr(nbr), 27, 0, n, _ffi.ptr(bt), 64,
                                                      _ffi.ptr(out), None, None, _ffi.ptr(part), 0,
                                                      _ffi.stream_of(out)), "gemm")
                e1.record()
                ts.append((e0, e1))
            torch.cuda.synchronize()
            us = sorted(1000 * a_.elapsed_time(b_) for a_, b_ in ts[5:])
            print(f"rows {n} pairs {pairs} mode {mode:2d} (arm {mode - 4 if mode >= 4 else '-'}): "
                  f"median {us[len(us) // 2]:.1f} us  min {us[0]:.1f}", flush=True)
        lib.rpc_spconv_gemm_bf16_mode(1)


if __name__ == "__main__":
    main()
