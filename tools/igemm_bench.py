"""Timing of the dense implicit-GEMM maps other than S1 (S2, its data gradient D2, the 1x1 P1 and the
2x2 stride-2 deconvolution U2 / its data gradient G2) at the shapes of the SECOND / SECONDFPN /
Anchor3DHead step (batch 6), HIP events on the launch stream, interleaved rounds over rpc_dense_tune
knob 2 variants. Prints per case the median / min µs, TFLOP/s and algorithmic GB/s (source image +
output image + weights, bf16)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from robustpointclouds_amd import _ffi  # noqa: E402

S2, D2, P1, U2, G2 = 1, 2, 3, 4, 5
B = 6
# (label, map, row image, source image, output image, ci, co, taps)
CASES = [
    ("S2 fwd 128->256", S2, (B, 100, 88), (B, 200, 176), (B, 100, 88), 128, 256, 9),
    ("D2 dgrad 256->128", D2, (B, 200, 176), (B, 100, 88), (B, 200, 176), 256, 128, 9),
    ("P1 deblock1 128->256", P1, (B, 200, 176), (B, 200, 176), (B, 200, 176), 128, 256, 1),
    ("P1 deblock1 dgrad 256->128", P1, (B, 200, 176), (B, 200, 176), (B, 200, 176), 256, 128, 1),
    ("U2 deblock2 256->256", U2, (B, 100, 88), (B, 100, 88), (B, 200, 176), 256, 256, 4),
    ("G2 deblock2 dgrad 256->256", G2, (B, 100, 88), (B, 200, 176), (B, 100, 88), 256, 256, 4),
    ("P1 head 512->128", P1, (B, 200, 176), (B, 200, 176), (B, 200, 176), 512, 128, 1),
    ("P1 head dgrad 128->512", P1, (B, 200, 176), (B, 200, 176), (B, 200, 176), 128, 512, 1),
]


def main(rounds=5, iters=10, variants=(0,), only=None):
    lib = _ffi.load()
    dev = torch.device("cuda")
    st = torch.cuda.current_stream()
    res = {}
    for (label, fmap, R, S, O, ci, co, taps) in CASES:
        if only and not any(o in label for o in only):
            continue
        ns, no, nr = S[0] * S[1] * S[2], O[0] * O[1] * O[2], R[0] * R[1] * R[2]
        x = (torch.rand(ns, ci, device=dev) * 2 - 1).to(torch.bfloat16)
        wt = ((torch.rand(taps, co, ci, device=dev) * 2 - 1) * 0.05).to(torch.bfloat16)
        z = torch.empty(no, co, dtype=torch.bfloat16, device=dev)
        ri, si, oi = _ffi.int_arr(R), _ffi.int_arr(S), _ffi.int_arr(O)
        part = torch.empty(lib.rpc_dense_conv_blocks(fmap, ri), 2 * co, device=dev)
        macs_per_row = ci * co * (taps if fmap in (S2, D2) else (4 if fmap == G2 else 1))
        rows = nr * (4 if fmap == U2 else 1)
        if fmap == D2:
            macs_per_row = ci * co * 9 / 4            # only the 1/2/2/4 live taps of a parity class
        flops = 2.0 * rows * macs_per_row
        nbytes = 2.0 * (ns * ci + no * co + taps * ci * co)

        def run():
            # data-gradient maps carry no BatchNorm partials (D2 then runs its parity-split form)
            _ffi.check(lib.rpc_dense_conv(fmap, _ffi.ptr(x), ci, ci, _ffi.ptr(wt), co, _ffi.ptr(z), co, 0, 0,
                                          None if fmap in (D2, G2) else _ffi.ptr(part), ri, si, oi,
                                          _ffi.stream_of(z)), "rpc_dense_conv")
        times = {v: [] for v in variants}
        ref = None
        for r in range(rounds):
            for v in variants:
                lib.rpc_dense_tune(2, v)
                run()
                if r == 0:
                    torch.cuda.synchronize()
                    if ref is None:
                        ref = (z.clone(), part.clone())
                    elif not (torch.equal(ref[0], z) and (fmap in (D2, G2) or torch.equal(ref[1], part))):
                        print(f"  {label}: variant {v} differs from variant {variants[0]}", flush=True)
                run()
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                e0.record(st)
                for _ in range(iters):
                    run()
                e1.record(st)
                e1.synchronize()
                times[v].append(e0.elapsed_time(e1) * 1e3 / iters)
        lib.rpc_dense_tune(2, 0)
        res[label] = {}
        for v in variants:
            t = sorted(times[v])
            med = t[len(t) // 2]
            res[label][f"v{v}"] = dict(med_us=round(med, 2), min_us=round(t[0], 2),
                                       tflops=round(flops / (med * 1e-6) / 1e12, 1),
                                       gbps=round(nbytes / (med * 1e-6) / 1e9, 0))
        print(label, json.dumps(res[label]), flush=True)
    return res


if __name__ == "__main__":
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="0")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    main(a.rounds, a.iters, tuple(int(v) for v in a.variants.split(",")),
         [s for s in a.only.split(",") if s] or None)
