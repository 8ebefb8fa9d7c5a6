"""Standalone timing of the sparse bf16 weight gradient (rpc_spconv_wgrad_bf16, slab reduction included) and of the
bf16 forward / data-gradient GEMMs on the rulebooks of one bench step: a training step runs with a KernelTimer that
records every sparse launch's neighbour table; each bf16 layer is then re-timed ALONE (random bf16 rows of the same
shapes, median of rounds), next to its in-step time from the same timer (which runs beside the other stream).

    python tools/spwg_bench.py [centerpoint|voxelnet] [ops=wgrad,fwd,dgrad,sdgrad]
Knob: RPC_SPWG_VARIANTS="0,1" times rpc_sparse_tune(1, v) per value (weight-gradient kernel variant)."""
import collections
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from robustpointclouds_amd import _ffi  # noqa: E402
from robustpointclouds_amd.sparse_encoder import KernelTimer  # noqa: E402
from robustpointclouds_amd.trainer import Trainer, make_kitti_model, make_nus_model  # noqa: E402


def r8(c):
    return (c + 7) // 8 * 8


def timeit(fn, iters=10, rounds=5):
    fn()
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(rounds):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            fn()
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3 / iters)
    return sorted(ts)[len(ts) // 2]


def main():
    model_name = sys.argv[1] if len(sys.argv) > 1 else "centerpoint"
    ops = (sys.argv[2] if len(sys.argv) > 2 else "wgrad").split(",")
    variants = [int(v) for v in os.environ.get("RPC_SPWG_VARIANTS", "0").split(",")]
    dev = torch.device("cuda")
    torch.manual_seed(0)
    if model_name == "centerpoint":
        model = make_nus_model(device=dev, epoch=3)
        data = bench._nus_batches(2, 4, 0, dev)
    else:
        model = make_kitti_model(num_classes=3, device=dev, epoch=3)
        data = bench._batches(2, 6, 0, dev, 3)
    tr = Trainer(model, bf16=True, device=dev)
    for i in range(3):
        tr.train_step(*data[i % 2], next_points=data[(i + 1) % 2][0])
    torch.cuda.synchronize()
    timer = KernelTimer()
    model.middle_encoder.timer = timer
    timer.enabled = True
    tr.train_step(*data[1], next_points=data[0][0])
    torch.cuda.synchronize()
    timer.enabled = False
    lib = _ffi.load()
    st = _ffi.stream_of(torch.empty(1, device=dev))
    tot = collections.defaultdict(float)
    for (e0, e1, nbr, ci, co, kname, dt) in timer.recs:
        if dt != "bf16":
            continue
        if "wgrad" in kname:
            op = "wgrad"
        elif "k_gemm_bf16" in kname:
            op = "fwd" if kname.rstrip(">").split(",")[2].strip() == "0" else "dgrad"
        else:
            continue
        if op not in ops and not (op == "fwd" and "sdgrad" in ops):
            continue
        instep = e0.elapsed_time(e1) * 1e3
        n_out, K = nbr.shape
        n_in = int(nbr.max().item()) + 1
        pairs = int((nbr >= 0).sum().item())
        fl = 2.0 * pairs * ci * co
        h = (torch.rand(n_in, r8(ci), device=dev) * 2 - 1).to(torch.bfloat16)
        dz = (torch.rand(n_out, r8(co), device=dev) * 2 - 1).to(torch.bfloat16)
        row = [f"{kname:42s} n_out {n_out:7d} pairs {pairs:8d} in-step {instep:7.1f} us"]
        if op == "wgrad":
            wsz = lib.rpc_spconv_wgrad_bf16_workspace_size(n_out, K, ci, co)
            ws = _ffi.workspace(wsz, dev)
            dW = torch.empty(K, ci, co, device=dev)
            for v in variants:
                lib.rpc_sparse_tune(1, v)

                def run():
                    _ffi.check(lib.rpc_spconv_wgrad_bf16(_ffi.ptr(h), ci, _ffi.ptr(nbr), K, n_out, _ffi.ptr(dz), co,
                                                         _ffi.ptr(dW), _ffi.ptr(ws), wsz, st), "wgrad")
                us = timeit(run)
                tot[v] += us
                row.append(f"v{v} {us:7.1f} us {fl / (us * 1e-6) / 1e12:6.1f} TF")
            lib.rpc_sparse_tune(1, 0)
        elif op == "fwd" and nbr.shape[0] != n_in and "sdgrad" in ops:
            # a strided layer: its data gradient runs on the input-side map nbr_in[i][k] = o (nbr[o][k] = i),
            # timed as is and with the input rows grouped by neighbour mask (stable sort: rows of one block then
            # share their few offsets — for stride 2 the coordinate parity decides which ones)
            o_idx, k_idx = torch.nonzero(nbr >= 0, as_tuple=True)
            nin = torch.full((n_in, K), -1, dtype=torch.int32, device=dev)
            nin[nbr[o_idx, k_idx].long(), k_idx] = o_idx.to(torch.int32)
            bits = (1 << torch.arange(K, device=dev, dtype=torch.int64))
            mask = ((nin >= 0).to(torch.int64) * bits).sum(1)
            nin_sorted = nin[torch.sort(mask, stable=True).indices].contiguous()
            NGP, KGP = (ci + 15) // 16 * 16, (co + 31) // 32 * 32
            a = (torch.rand(n_out, r8(co), device=dev) * 2 - 1).to(torch.bfloat16)
            bt = (torch.rand(K, NGP, KGP, device=dev) * 0.1).to(torch.bfloat16)
            out = torch.empty(n_in, ci, device=dev)
            for tag, mp in (("as is", nin), ("mask-sorted", nin_sorted)):
                def run():
                    _ffi.check(lib.rpc_spconv_gemm_bf16_n(_ffi.ptr(a), n_out, co, _ffi.ptr(mp), K, 0, n_in, _ffi.ptr(bt),
                                                          ci, _ffi.ptr(out), None, None, None, 2, st), "gemm")
                us = timeit(run)
                tot["sdgrad " + tag] += us
                row.append(f"dgrad {tag} {us:7.1f} us")
            print("  ".join(row).replace("in-step", "(fwd in-step)"), flush=True)
            continue
        else:
            # the GEMM core on this rulebook, plain epilogue (submanifold layers: map = nbr, the data gradient
            # reads it reversed; strided layers: see sdgrad)
            if nbr.shape[0] != n_in or op not in ops:
                continue
            kg, ng = (ci, co) if op == "fwd" else (co, ci)
            NGP, KGP = (ng + 15) // 16 * 16, (kg + 31) // 32 * 32
            a = (torch.rand(n_out, r8(kg), device=dev) * 2 - 1).to(torch.bfloat16)
            bt = (torch.rand(K, NGP, KGP, device=dev) * 0.1).to(torch.bfloat16)
            out = torch.empty(n_out, ng, device=dev)
            rev = 0 if op == "fwd" else 1

            def run():
                _ffi.check(lib.rpc_spconv_gemm_bf16_n(_ffi.ptr(a), n_out, kg, _ffi.ptr(nbr), K, rev, n_out, _ffi.ptr(bt), ng,
                                                      _ffi.ptr(out), None, None, None, 2, st), "gemm")
            us = timeit(run)
            tot[op] += us
            row.append(f"v0 {us:7.1f} us {fl / (us * 1e-6) / 1e12:6.1f} TF (plain epilogue)")
        print("  ".join(row), flush=True)
    print("total standalone us per variant / op:", {k: round(v, 1) for k, v in tot.items()}, flush=True)


if __name__ == "__main__":
    main()
