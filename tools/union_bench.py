"""Microbenchmark: the sparse 16-bit GEMM with and without the per-block source-row unions on the metric's
rulebooks (synthetic KITTI 3-class batch of 6 frames): per layer the union sizes (mean / p99 / share of blocks
past the kernel's LDS capacity) and the HIP-event time of the forward and data-gradient GEMMs both ways."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from robustpointclouds_amd import _ffi, voxelize  # noqa: E402
from robustpointclouds_amd import sparse_encoder as se  # noqa: E402
from robustpointclouds_amd.synthetic import KITTI_PC_RANGE, KITTI_VOXEL_SIZE, kitti_batch  # noqa: E402

dev = torch.device("cuda")
lib = _ffi.load()
pts, _, _ = kitti_batch(6, seed0=0, num_classes=3)
pts = [torch.from_numpy(p).to(dev) for p in pts]
d = voxelize.Voxelization(KITTI_VOXEL_SIZE, KITTI_PC_RANGE, 5, 16000).to(dev).voxelize_frames(pts)
coors = d["coors"].to(torch.int32).contiguous()
enc = se.SparseEncoder(4, [41, 1600, 1408]).to(dev)
enc.bf16 = True
plan = se._RulebookPlan(lib, enc, coors, coors.shape[0], 6, dev)
torch.cuda.synchronize()


def timeit(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1000.0


def r8(c):
    return (c + 7) // 8 * 8


cap = {32: 512, 64: 512, 128: 224}
for li, sp in enumerate(enc.specs):
    p = plan.get(li)
    if li == 0:
        continue
    for direction in ("fwd", "dgrad"):
        if direction == "fwd":
            nbr, un, rev, n_rows, n_src, kg, ng = p["nbr"], p["un"], 0, p["n_out"], p["n_in"], sp.ci, sp.co
        else:
            if sp.kind == "subm":
                nbr, un, rev = p["nbr"], p["un"], 1
            else:
                nbr, un, rev = p["nbr_in"], p["un_in"], 0
            n_rows, n_src, kg, ng = p["n_in"], p["n_out"], sp.co, sp.ci
        uc = un.ucnt.cpu().numpy()
        kgp = (kg + 31) // 32 * 32
        over = float((uc > cap[kgp]).mean())
        valid = float((nbr >= 0).sum()) / max(n_rows, 1)
        a = torch.randn((n_src, r8(kg)), device=dev).to(torch.bfloat16)
        W = torch.randn((sp.K, kg, ng), device=dev) * 0.1
        bt = torch.empty(lib.rpc_spconv_bf16_weight_elems(sp.K, kg, ng, 0), dtype=torch.bfloat16, device=dev)
        st = _ffi.stream_of(W)
        _ffi.check(lib.rpc_spconv_prep_weight_bf16(_ffi.ptr(W), sp.K, kg, ng, 0, _ffi.ptr(bt), st), "prep")
        out = torch.empty((n_rows, ng), device=dev)
        part = torch.empty((max(lib.rpc_spconv_gemm_blocks(n_rows), 1), 2 * ng), device=dev)
        ez = torch.randn((n_rows, ng), device=dev)
        ebn = torch.rand(4 * ng, device=dev) + 0.5
        epi = 0 if direction == "fwd" else 1

        def run(u):
            _ffi.check(lib.rpc_spconv_gemm_ex(_ffi.ptr(a), 0, n_src, kg, _ffi.ptr(nbr), sp.K, rev,
                                              _ffi.C.byref(u.c) if u is not None else None, n_rows, _ffi.ptr(bt), ng,
                                              _ffi.ptr(out), _ffi.ptr(ez) if epi else None,
                                              _ffi.ptr(ebn) if epi else None, _ffi.ptr(part), epi, st), "gemm")
        t0 = timeit(lambda: run(None))
        t1 = timeit(lambda: run(un))
        nb = max(lib.rpc_rulebook_union_blocks(n_rows), 1)
        dbg = torch.zeros((nb, 8), dtype=torch.int64, device=dev)
        lib.rpc_spconv_gemm_debug(_ffi.C.c_void_p(dbg.data_ptr()))
        run(un)
        torch.cuda.synchronize()
        lib.rpc_spconv_gemm_debug(None)
        dd = dbg.cpu().numpy().astype(np.float64)
        ok = dd[:, 5] > 0
        pro = (dd[ok, 1] - dd[ok, 0]).mean()
        loop = (dd[ok, 2] - dd[ok, 1]).mean()
        nk = dd[ok, 3].mean()
        span = (dd[:, 2].max() - dd[:, 0].min())
        print(f"L{li:2d} {sp.kind:5s} {direction:5s} {kg:3d}->{ng:3d} rows {n_rows:7d} valid/row {valid:5.2f} "
              f"U mean {uc.mean():6.1f} p99 {np.percentile(uc, 99):6.0f} over {over:5.3f} | "
              f"regular {t0:7.1f} us  union {t1:7.1f} us | clk: prologue+gather {pro:7.0f} loop {loop:7.0f} "
              f"({loop / max(nk, 1):5.0f}/step, {nk:4.1f} steps) span {span:8.0f}", flush=True)
