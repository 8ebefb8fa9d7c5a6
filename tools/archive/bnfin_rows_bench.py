"""rpc_bn_finalize timing alone (fp32 partial rows, mode 0 and 1) over channel counts and partial-row counts,
HIP-event us per call, median of rounds; A/B with RPC_BN_FIN_WIDE=0 in a second process.

    python tools/bnfin_bench.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from robustpointclouds_amd import _ffi  # noqa: E402


def main():
    lib = _ffi.load()
    dev = torch.device("cuda")
    for C in (16, 32, 64, 128):
        for nblk in (512, 1500, 3000, 6000):
            part = torch.rand(nblk, 2 * C, device=dev)
            g, b = torch.ones(C, device=dev), torch.zeros(C, device=dev)
            rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
            fbn = torch.rand(4 * C, device=dev)
            out = torch.empty(5 * C, device=dev)
            dg, db = torch.empty(C, device=dev), torch.empty(C, device=dev)
            st = _ffi.stream_of(part)
            res = []
            for mode in (0, 1):
                def run():
                    _ffi.check(lib.rpc_bn_finalize(_ffi.ptr(part), nblk, C, 64 * nblk, mode, _ffi.ptr(g), _ffi.ptr(b),
                                                   1e-3, 0.01, _ffi.ptr(rm), _ffi.ptr(rv), _ffi.ptr(fbn), _ffi.ptr(out),
                                                   _ffi.ptr(dg), _ffi.ptr(db), None, st), "rpc_bn_finalize")
                for _ in range(3):
                    run()
                ts = []
                for _ in range(5):
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for _ in range(20):
                        run()
                    e1.record()
                    e1.synchronize()
                    ts.append(e0.elapsed_time(e1) * 1e3 / 20)
                res.append(sorted(ts)[2])
            print(f"C {C:4d} rows {nblk:5d}  mode0 {res[0]:6.2f} us  mode1 {res[1]:6.2f} us", flush=True)


if __name__ == "__main__":
    main()
