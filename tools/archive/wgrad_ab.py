"""Isolated S1 weight-gradient timing per rpc_dense_tune knob 1 value (0 = k_wgrad_s1, 1 = k_wgrad,
2 = k_wgrad_s1 pipelined) at the SECOND shapes, slab reduction included, median of rounds."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from robustpointclouds_amd import _ffi  # noqa: E402

SHAPES = [(6, 200, 176, 128, 128), (6, 100, 88, 256, 256), (6, 200, 176, 128, 256)]


def main(rounds=5, iters=10):
    lib = _ffi.load()
    dev = torch.device("cuda")
    st = torch.cuda.current_stream()
    vals = [int(v) for v in os.environ.get("VALS", "0,2").split(",")]
    for (B, H, W, ci, co) in SHAPES:
        x = (torch.rand(B * H * W, ci, device=dev) * 2 - 1).to(torch.bfloat16)
        dz = (torch.rand(B * H * W, co, device=dev) * 2 - 1).to(torch.bfloat16)
        img = _ffi.int_arr((B, H, W))
        wsz = lib.rpc_dense_wgrad_workspace_size(0, img, ci, co)
        ws = _ffi.workspace(wsz, dev)
        dW = torch.empty(co, ci, 3, 3, device=dev)
        times = {v: [] for v in vals}
        for r in range(rounds):
            for v in vals:
                lib.rpc_dense_tune(1, v)

                def run():
                    _ffi.check(lib.rpc_dense_wgrad(0, 0, _ffi.ptr(x), ci, ci, _ffi.ptr(dz), co, co, img, img, img,
                                                   _ffi.ptr(dW), _ffi.ptr(ws), wsz, _ffi.stream_of(dW)), "wgrad")
                run(); run()
                e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
                e0.record(st)
                for _ in range(iters):
                    run()
                e1.record(st)
                e1.synchronize()
                times[v].append(e0.elapsed_time(e1) * 1e3 / iters)
        lib.rpc_dense_tune(1, 0)
        fl = 2.0 * B * H * W * ci * co * 9
        print(f"B{B} {H}x{W} {ci}->{co}", json.dumps({f"knob1={v}": {"us": round(sorted(t)[len(t) // 2], 2),
              "tflops": round(fl / (sorted(t)[len(t) // 2] * 1e-6) / 1e12, 1)} for v, t in times.items()}), flush=True)


if __name__ == "__main__":
    main()
