"""Micro-benchmark of rpc_bn_finalize (52 calls per KITTI step): clean vs dirty L2 before each call."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from robustpointclouds_amd import _ffi

dev = torch.device("cuda")
lib = _ffi.load()
st = _ffi.stream_of(torch.empty(1, device=dev))
for nblk, C in ((858, 128), (252, 256), (2000, 64), (300, 16)):
    part = torch.randn(nblk, 2 * C, device=dev)
    gamma, beta = torch.ones(C, device=dev), torch.zeros(C, device=dev)
    rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
    bn = torch.empty(4 * C, device=dev)
    ws = None   # rpc_bn_finalize needs no workspace since r01 v11
    big = torch.empty(256 << 20, dtype=torch.uint8, device=dev)
    call = lambda: lib.rpc_bn_finalize(_ffi.ptr(part), nblk, C, nblk * 64, 0, _ffi.ptr(gamma), _ffi.ptr(beta), 1e-3,
                                       0.01, _ffi.ptr(rm), _ffi.ptr(rv), None, _ffi.ptr(bn), None, None, _ffi.ptr(ws), st)
    for dirty in (False, True):
        for _ in range(3):
            call()
        torch.cuda.synchronize()
        tot = 0.0
        for _ in range(20):
            if dirty:
                big.fill_(1)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            call()
            e1.record()
            torch.cuda.synchronize()
            tot += e0.elapsed_time(e1)
        print(f"nblk={nblk} C={C} dirty={dirty}: {tot / 20 * 1000:.1f} us", flush=True)
