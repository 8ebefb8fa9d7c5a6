"""A/B timing of the dense BatchNorm elementwise passes (rpc_dense_bn_apply, rpc_dense_bnbwd_apply) over the
row mappings of rpc_dense_tune knob 9 (0: contiguous row chunks per block, default; 1: the former grid-stride batches), interleaved rounds in one process, HIP events on the launch stream; checks
that every variant writes the same bits. Prints per shape and variant the median µs and GB/s of algorithmic bytes
(bn_apply: z read + h write; bnbwd_apply: dh + z read, dz write; bf16)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from robustpointclouds_amd import _ffi  # noqa: E402

SHAPES = [(6 * 200 * 176, 128), (6 * 100 * 88, 256), (6 * 200 * 176, 256)]


def main(rounds=7, iters=20, variants=(1, 0)):
    lib = _ffi.load()
    dev = torch.device("cuda")
    st = torch.cuda.current_stream()
    for (M, C) in SHAPES:
        z = torch.randn(M, C, device=dev).to(torch.bfloat16)
        dh = torch.randn(M, C, device=dev).to(torch.bfloat16)
        bn = torch.cat([torch.rand(C) + 0.5, torch.randn(C) * 0.2, torch.randn(C) * 0.1, torch.rand(C) + 0.5]).to(dev)
        bnb = torch.cat([torch.rand(C) + 0.5, torch.randn(C) * 0.1, torch.randn(C) * 0.1, torch.randn(C) * 0.1,
                         torch.rand(C) + 0.5]).to(dev)
        h = torch.empty(M, C, dtype=torch.bfloat16, device=dev)
        dz = torch.empty(M, C, dtype=torch.bfloat16, device=dev)
        s = _ffi.stream_of(z)

        def fwd():
            _ffi.check(lib.rpc_dense_bn_apply(_ffi.ptr(z), M, C, _ffi.ptr(bn), _ffi.ptr(h), C, 0, s), "bn_apply")

        def bwd():
            _ffi.check(lib.rpc_dense_bnbwd_apply(_ffi.ptr(dh), C, 0, _ffi.ptr(z), M, C, _ffi.ptr(bn), _ffi.ptr(bnb),
                                                 _ffi.ptr(dz), s), "bnbwd_apply")

        res = {}
        outs = {}
        for name, fn, nbytes in (("bn_apply", fwd, 4 * M * C), ("bnbwd_apply", bwd, 6 * M * C)):
            times = {v: [] for v in variants}
            for r in range(rounds):
                for v in variants:
                    old = lib.rpc_dense_tune(9, v)
                    fn()
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(st)
                    for _ in range(iters):
                        fn()
                    e1.record(st)
                    e1.synchronize()
                    times[v].append(e0.elapsed_time(e1) * 1e3 / iters)
                    if r == 0:
                        outs[(name, v)] = (h if name == "bn_apply" else dz).clone()
                    lib.rpc_dense_tune(9, old)
            for v in variants:
                assert torch.equal(outs[(name, v)], outs[(name, variants[0])]), (name, v)
                t = sorted(times[v])[rounds // 2]
                res[f"{name} v{v}"] = dict(med_us=round(t, 2), gbps=round(nbytes / (t * 1e-6) / 1e9, 0))
        print(f"M={M} C={C}", json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
