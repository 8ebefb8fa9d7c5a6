"""Do the CenterHead's per-task 64-channel convolutions gain from running side by side? Six 3x3 64 -> 64 S1
convs at batch 4 x 128 x 128 (one per nuScenes task, each with its own input and weights) on the bf16 dense
engine: (a) one after another on one stream (the current head), (b) spread over 2 / 3 / 6 streams, (c) as one
launch of batch 24 (the same work as a single grid: what a task-grouped launch would cost). HIP-event us.

    python tools/head_conc_bench.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from robustpointclouds_amd import _ffi  # noqa: E402
from robustpointclouds_amd import dense_bev as db  # noqa: E402


def main():
    dev = torch.device("cuda")
    lib = _ffi.load()
    eng = db._Eng(lib, False)
    B, H, W, C, T = 4, 128, 128, 64, 6
    xs = [db._image(B, C, H, W, dev).normal_() for _ in range(T)]
    ws = [(torch.randn(9, C, C, device=dev) * 0.05).to(torch.bfloat16) for _ in range(T)]
    zs = [db._image(B, C, H, W, dev) for _ in range(T)]
    xbig = db._image(B * T, C, H, W, dev).normal_()
    zbig = db._image(B * T, C, H, W, dev)
    R = _ffi.int_arr((B, H, W))
    RB = _ffi.int_arr((B * T, H, W))

    def conv(x, w, z, st, r=R):
        _ffi.check(eng.conv(db.S1, _ffi.ptr(x), C, C, _ffi.ptr(w), C, _ffi.ptr(z), C, 0, 0, None, r, r, r, st), "conv")

    main_s = torch.cuda.current_stream()
    streams = [torch.cuda.Stream() for _ in range(T)]

    def serial():
        st = _ffi.stream_of(xs[0])
        for t in range(T):
            conv(xs[t], ws[t], zs[t], st)

    def spread(ns):
        def f():
            ev = torch.cuda.Event()
            ev.record(main_s)
            for t in range(T):
                s = streams[t % ns]
                s.wait_event(ev)
                with torch.cuda.stream(s):
                    conv(xs[t], ws[t], zs[t], s.cuda_stream)
            for s in streams[:ns]:
                e = torch.cuda.Event()
                e.record(s)
                main_s.wait_event(e)
        return f

    def grouped():
        conv(xbig, ws[0], zbig, main_s.cuda_stream, RB)

    def timeit(fn, iters=20, rounds=5):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(rounds):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(main_s)
            for _ in range(iters):
                fn()
            e1.record(main_s)
            e1.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3 / iters)
        return sorted(ts)[len(ts) // 2]

    print(f"6 x conv 64->64 at {B}x{H}x{W}: serial {timeit(serial):.1f} us, 2 streams {timeit(spread(2)):.1f} us, "
          f"3 streams {timeit(spread(3)):.1f} us, 6 streams {timeit(spread(6)):.1f} us, one batch-24 launch "
          f"{timeit(grouped):.1f} us", flush=True)


if __name__ == "__main__":
    main()
