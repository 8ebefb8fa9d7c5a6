"""S1 weight-gradient timing (rpc_dense_wgrad, its slab reduce included) on the metric's SECOND shapes, per
rpc_dense_tune knob-1 variant: 4 = k_wgrad_s1 (row segments, 3 taps per block), 3 = k_wgrad_s1c (column walk,
9 taps per block; the default 0 since r06). HIP-event us per call, median of rounds.

    python tools/s1wg_bench.py [variants...]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from robustpointclouds_amd import _ffi  # noqa: E402
from tools.dwg_bench import timeit  # noqa: E402

S1 = 0
SHAPES = [("200x176 256->128", (6, 200, 176), 256, 128, 1), ("200x176 128->128", (6, 200, 176), 128, 128, 5),
          ("100x88 256->256", (6, 100, 88), 256, 256, 5)]


def main():
    variants = sys.argv[1:] or ["4", "3"]   # "v" or "v:seg" or "v:seg:dbg" (knobs 6 / 7: k_wgrad_s1c segment, arms)
    lib = _ffi.load()
    dev = torch.device("cuda")
    tot = {v: 0.0 for v in variants}
    for name, r, ci, co, n in SHAPES:
        M = r[0] * r[1] * r[2]
        x = (torch.rand(M, ci, device=dev) * 2 - 1).to(torch.bfloat16)
        dz = (torch.rand(M, co, device=dev) * 2 - 1).to(torch.bfloat16)
        R = _ffi.int_arr(r)
        wsz = lib.rpc_dense_wgrad_workspace_size(S1, R, ci, co)
        ws = _ffi.workspace(wsz, dev)
        dW = torch.empty(co, ci, 3, 3, device=dev)
        st = _ffi.stream_of(dW)
        row = []
        for v in variants:
            kv, _, rest = v.partition(":")
            seg, _, dbg = rest.partition(":")
            old = lib.rpc_dense_tune(1, int(kv))
            old6 = lib.rpc_dense_tune(6, int(seg or 0))
            old7 = lib.rpc_dense_tune(7, int(dbg or 0))

            def run():
                _ffi.check(lib.rpc_dense_wgrad(S1, 0, _ffi.ptr(x), ci, ci, _ffi.ptr(dz), co, co, R, R, R, _ffi.ptr(dW),
                                               _ffi.ptr(ws), wsz, st), "wgrad")
            us = timeit(run)
            lib.rpc_dense_tune(1, old)
            lib.rpc_dense_tune(6, old6)
            lib.rpc_dense_tune(7, old7)
            tot[v] += us * n
            fl = 2.0 * M * ci * co * 9
            row.append(f"v{v} {us:7.1f} us ({fl / us / 1e6:6.0f} TFLOP/s)")
        print(f"{name:20s} x{n}: " + "  ".join(row), flush=True)
    print("per step (11 launches): " + "  ".join(f"v{v} {t / 1e3:.3f} ms" for v, t in tot.items()))


if __name__ == "__main__":
    main()
