"""Probe: how much of k_gemm_bf16's time the MFMA rows without a neighbour cost. The same 64 -> 64 / 32 -> 32
rulebooks of a synthetic KITTI batch, timed as they come and with their rows visited in neighbour-mask order
within windows of W rows (rows physically permuted here; a kernel with a permutation would write each row in
place — the per-row results are the same). HIP-event median per launch.
    python tools/spgemm_sort_probe.py"""
import sys

import numpy as np
import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from robustpointclouds_amd import _ffi, voxelize  # noqa: E402
from robustpointclouds_amd.sparse_encoder import SparseEncoder  # noqa: E402
from robustpointclouds_amd.synthetic import KITTI_PC_RANGE, KITTI_VOXEL_SIZE, kitti_batch  # noqa: E402


def _time(lib, a, n, ci, co, nbr, bt, rev, reps=25):
    out = torch.empty((n, co), device=a.device)
    part = torch.empty((lib.rpc_spconv_gemm_blocks(n), 2 * co), device=a.device)
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        _ffi.check(lib.rpc_spconv_gemm_bf16_n(_ffi.ptr(a), a.shape[0], ci, _ffi.ptr(nbr), nbr.shape[1], rev, n,
                                              _ffi.ptr(bt), co, _ffi.ptr(out), None, None, _ffi.ptr(part), 0,
                                              _ffi.stream_of(out)), "gemm")
        e1.record()
        ts.append((e0, e1))
    torch.cuda.synchronize()
    us = sorted(1000 * x.elapsed_time(y) for x, y in ts[5:])
    return us[len(us) // 2]


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
    seen = set()
    for nbr, ci, co in enc.flop_probe[-1]:
        if nbr.data_ptr() in seen or ci < 16:
            continue
        seen.add(nbr.data_ptr())
        n, K = nbr.shape
        a = torch.randn((max(n, 200000), ci), device=dev).to(torch.bfloat16)
        W = torch.randn((K, ci, co), device=dev) * 0.05
        bt = torch.empty(lib.rpc_spconv_bf16_weight_elems(K, ci, co, 0), dtype=torch.bfloat16, device=dev)
        _ffi.check(lib.rpc_spconv_prep_weight_bf16(_ffi.ptr(W), K, ci, co, 0, _ffi.ptr(bt), _ffi.stream_of(W)), "prep")
        nb = nbr.cpu().numpy()
        mask = ((nb >= 0).astype(np.int64) << np.arange(K)).sum(1)
        line = f"rows {n:7d} K {K:2d} {ci:3d}->{co:3d} pairs {int((nb >= 0).sum()):8d}: as built {_time(lib, a, n, ci, co, nbr, bt, 0):6.1f} us"
        for W_ in (256, 2048, 8192):
            order = np.concatenate([s + np.argsort(mask[s:s + W_], kind="stable") for s in range(0, n, W_)])
            ns = torch.from_numpy(nb[order]).to(dev).contiguous()
            line += f" | sorted/{W_} {_time(lib, a, n, ci, co, ns, bt, 0):6.1f}"
        print(line, flush=True)


if __name__ == "__main__":
    main()
