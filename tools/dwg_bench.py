"""Dense weight-gradient timing (rpc_dense_wgrad, reduce included) on the step's non-S1 / narrow shapes: the 3-class
SECOND / FPN strided, 1x1 and transposed convs and the CenterPoint head's 64-channel convs. HIP-event us, median
of rounds; A/B two builds with RPC_HIP_LIB.

    python tools/dwg_bench.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from robustpointclouds_amd import _ffi  # noqa: E402

S1, S2, P1, U2 = 0, 1, 3, 4
# (name, map, (B, H, W) of the row image, (B, H, W) source, (B, H, W) output, ci, co)
SHAPES = [
    ("3class S2 128->256", S2, (6, 100, 88), (6, 200, 176), (6, 100, 88), 128, 256),
    ("3class P1 128->256", P1, (6, 200, 176), (6, 200, 176), (6, 200, 176), 128, 256),
    ("3class U2 256->256", U2, (6, 100, 88), (6, 100, 88), (6, 200, 176), 256, 256),
    ("3class head P1 512->128", P1, (6, 200, 176), (6, 200, 176), (6, 200, 176), 512, 128),
    ("CP head S1 64->64", S1, (4, 128, 128), (4, 128, 128), (4, 128, 128), 64, 64),
    ("CP head S1 64->320", S1, (4, 128, 128), (4, 128, 128), (4, 128, 128), 64, 320),
    ("CP head S1 320->64", S1, (4, 128, 128), (4, 128, 128), (4, 128, 128), 320, 64),
]


def timeit(fn, iters=20, rounds=5):
    for _ in range(3):
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
    lib = _ffi.load()
    dev = torch.device("cuda")
    tot = 0.0
    for name, mp, r, s_, o, ci, co in SHAPES:
        xs = s_ if mp != U2 else r
        x = (torch.rand(xs[0] * xs[1] * xs[2], ci, device=dev) * 2 - 1).to(torch.bfloat16)
        ds = o if mp != U2 else o
        dz = (torch.rand(ds[0] * ds[1] * ds[2], co, device=dev) * 2 - 1).to(torch.bfloat16)
        R, S, O = _ffi.int_arr(r), _ffi.int_arr(s_), _ffi.int_arr(o)
        wsz = lib.rpc_dense_wgrad_workspace_size(mp, R, ci, co)
        ws = _ffi.workspace(wsz, dev)
        T = 9 if mp in (S1, S2) else (4 if mp == U2 else 1)
        dW = torch.empty(co, ci, T, device=dev)
        st = _ffi.stream_of(dW)

        def run():
            _ffi.check(lib.rpc_dense_wgrad(mp, 0, _ffi.ptr(x), ci, ci, _ffi.ptr(dz), co, co, R, S, O, _ffi.ptr(dW),
                                           _ffi.ptr(ws), wsz, st), "rpc_dense_wgrad")
        us = timeit(run)
        tot += us
        print(f"{name:26s} {us:8.1f} us", flush=True)
    print(f"total {tot:.1f} us", flush=True)


if __name__ == "__main__":
    main()
