"""The sparse BatchNorm-backward row producer (rpc_bnbwd_to_bf16_rows: fp32 dy + z rows -> bf16 dz rows) alone at
the CenterPoint and 3-class layer shapes: HIP-event us and effective GB/s (10 B per element: dy, z read, dz written).

    python tools/dz_bench.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from robustpointclouds_amd import _ffi  # noqa: E402

SHAPES = [(360000, 16), (593721, 32), (457070, 64), (183364, 128), (132053, 32), (106578, 64)]


def main():
    lib = _ffi.load()
    dev = torch.device("cuda")
    for n, c in SHAPES:
        dy = torch.randn(n, c, device=dev)
        z = torch.randn(n, c, device=dev)
        bnb = torch.cat([torch.rand(c, device=dev) + 0.5, torch.randn(c, device=dev) * 0.1,
                         torch.randn(c, device=dev) * 0.1, torch.randn(c, device=dev) * 0.1,
                         torch.rand(c, device=dev) + 0.5])
        dz = torch.empty(n, (c + 7) // 8 * 8, dtype=torch.bfloat16, device=dev)
        st = _ffi.stream_of(dz)

        def run():
            _ffi.check(lib.rpc_bnbwd_to_bf16_rows(_ffi.ptr(dy), _ffi.ptr(z), _ffi.ptr(bnb), n, c, _ffi.ptr(dz), st),
                       "dz")
        for _ in range(3):
            run()
        torch.cuda.synchronize()
        ts = []
        for _ in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                run()
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3 / 20)
        us = sorted(ts)[2]
        print(f"n {n:7d} c {c:4d}: {us:7.1f} us  {10.0 * n * c / (us * 1e-6) / 1e9:7.0f} GB/s", flush=True)


if __name__ == "__main__":
    main()
