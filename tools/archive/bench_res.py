"""Micro-benchmark: rpc_sparse_res_backward / _forward_h16 in isolation (HIP events)."""
import sys

import torch

sys.path.insert(0, ".")
from robustpointclouds_amd import _ffi  # noqa: E402

lib = _ffi.load()
dev = torch.device("cuda")
st = _ffi.stream_of(torch.empty(1, device=dev))
for n, c in ((360000, 16), (250000, 32), (150000, 64), (60000, 128)):
    t = lambda: torch.randn(n, c, device=dev)
    g1, g2, out, z = t(), t(), t().relu(), t()
    bn = torch.rand(4 * c, device=dev) + 0.5
    m = torch.empty(n, c, device=dev)
    part = torch.empty((n + 63) // 64, 2 * c, device=dev)
    hb = torch.empty(n, c, dtype=torch.float16, device=dev)
    hb2 = torch.empty(n, c, dtype=torch.bfloat16, device=dev)
    res = t()
    for name, fn in (("bwd", lambda: lib.rpc_sparse_res_backward(_ffi.ptr(g1), _ffi.ptr(g2), _ffi.ptr(out), _ffi.ptr(z),
                                                                  _ffi.ptr(bn), n, c, _ffi.ptr(m), _ffi.ptr(part), st)),
                     ("fwd", lambda: lib.rpc_sparse_res_forward_h16(_ffi.ptr(z), _ffi.ptr(bn), _ffi.ptr(res), n, c,
                                                                     _ffi.ptr(out), _ffi.ptr(hb), 1, _ffi.ptr(hb2), st))):
        for _ in range(3):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            fn()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / 20 * 1e3
        byts = n * c * 4 * (5 if name == "bwd" else 3) + (n * c * 4 if name == "fwd" else 0)
        print(f"{name} n={n} c={c}: {us:.1f} us, {byts / us / 1e3:.0f} GB/s")
