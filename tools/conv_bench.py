"""A/B timing of the S1 (3x3 stride-1) dense-conv kernels at the SECOND config shapes, interleaved
rounds in one process (rpc_dense_tune knob 0: 0 = by shape, 1 = k_conv3x3, 2 = k_conv3x3w; or --knob 5: k_conv3x3's
channels per block, 1 = 64, 2 = 32), HIP events on the
launch stream. Prints per shape and variant the median / min µs and TFLOP/s (2*B*H*W*ci*co*9)."""
import json
import sys

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from robustpointclouds_amd import _ffi  # noqa: E402

SHAPES = [(6, 200, 176, 128, 128), (6, 200, 176, 256, 128), (6, 200, 176, 128, 256), (6, 100, 88, 256, 256)]


def main(rounds=5, iters=10, variants=(0, 1, 2), shapes=None, knob=0, bnbwd=False):
    lib = _ffi.load()
    dev = torch.device("cuda")
    st = torch.cuda.current_stream()
    res = {}
    for (B, H, W, ci, co) in (shapes or SHAPES):
        x = (torch.rand(B * H * W, ci, device=dev) * 2 - 1).to(torch.bfloat16)
        wt = ((torch.rand(9, co, ci, device=dev) * 2 - 1) * 0.05).to(torch.bfloat16)
        z = torch.empty(B * H * W, co, dtype=torch.bfloat16, device=dev)
        img = _ffi.int_arr((B, H, W))
        nblk = lib.rpc_dense_conv_blocks(0, img)
        part = torch.empty(nblk, 2 * co, device=dev)
        zb = torch.randn(B * H * W, co, device=dev).to(torch.bfloat16)
        bnp = torch.cat([torch.rand(co) + 0.5, torch.randn(co) * 0.2, torch.randn(co) * 0.1,
                         torch.rand(co) + 0.5]).to(dev)

        def launch():
            if bnbwd:   # the data gradient with the fused BatchNorm-backward sums of the layer it enters
                _ffi.check(lib.rpc_dense_conv_bnbwd(_ffi.ptr(x), ci, ci, _ffi.ptr(wt), co, _ffi.ptr(z), co, _ffi.ptr(zb),
                                                    _ffi.ptr(bnp), _ffi.ptr(part), img, _ffi.stream_of(z)), "bnbwd")
            else:
                lib.rpc_dense_conv(0, _ffi.ptr(x), ci, ci, _ffi.ptr(wt), co, _ffi.ptr(z), co, 0, 0, _ffi.ptr(part),
                                   img, img, img, _ffi.stream_of(z))
        flops = 2.0 * B * H * W * ci * co * 9
        times = {v: [] for v in variants}
        for r in range(rounds):
            for v in variants:
                lib.rpc_dense_tune(knob, v)
                for _ in range(2):
                    launch()
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                e0.record(st)
                for _ in range(iters):
                    launch()
                e1.record(st)
                e1.synchronize()
                times[v].append(e0.elapsed_time(e1) * 1e3 / iters)
        lib.rpc_dense_tune(knob, 0)
        key = f"B{B} {H}x{W} {ci}->{co}"
        res[key] = {}
        for v in variants:
            t = sorted(times[v])
            res[key][f"v{v}"] = dict(med_us=round(t[len(t) // 2], 2), min_us=round(t[0], 2),
                                     tflops=round(flops / (t[len(t) // 2] * 1e-6) / 1e12, 1))
        print(key, json.dumps(res[key]), flush=True)
    return res


if __name__ == "__main__":
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="0,1,2")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--knob", type=int, default=0, help="rpc_dense_tune knob the variants set (0 or 5)")
    ap.add_argument("--shapes", default="", help="B,H,W,ci,co;... (default: the SECOND config shapes)")
    ap.add_argument("--bnbwd", action="store_true", help="time rpc_dense_conv_bnbwd (fused BN-backward sums)")
    a = ap.parse_args()
    shapes = [tuple(int(x) for x in sh.split(",")) for sh in a.shapes.split(";") if sh] or None
    main(a.rounds, a.iters, tuple(int(v) for v in a.variants.split(",")), shapes, a.knob, a.bnbwd)
