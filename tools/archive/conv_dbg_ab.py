"""Timing attribution of k_conv3x3x (rpc_dense_tune knob 4): the real kernel, without MFMAs, without operand
reads, and with neither (DMA + barriers only), at the SECOND shapes. Outputs of the debug arms are garbage."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from robustpointclouds_amd import _ffi  # noqa: E402

SHAPES = [(6, 200, 176, 128, 128), (6, 200, 176, 128, 256)]


def main(rounds=5, iters=10):
    lib = _ffi.load()
    dev = torch.device("cuda")
    st = torch.cuda.current_stream()
    shapes = [tuple(int(v) for v in t.split(",")) for t in os.environ["SHAPES"].split(";")] if os.environ.get("SHAPES") else SHAPES
    if os.environ.get("VARIANT"):
        lib.rpc_dense_tune(0, int(os.environ["VARIANT"]))
    for (B, H, W, ci, co) in shapes:
        x = (torch.rand(B * H * W, ci, device=dev) * 2 - 1).to(torch.bfloat16)
        wt = ((torch.rand(9, co, ci, device=dev) * 2 - 1) * 0.05).to(torch.bfloat16)
        z = torch.empty(B * H * W, co, dtype=torch.bfloat16, device=dev)
        img = _ffi.int_arr((B, H, W))
        part = torch.empty(lib.rpc_dense_conv_blocks(0, img), 2 * co, device=dev)
        dbgs = [int(v) for v in os.environ.get("DBGS", "0,1,17,64,65,81").split(",")]
        times = {d: [] for d in dbgs}
        for r in range(rounds):
            for d in times:
                lib.rpc_dense_tune(4, d)
                def run():
                    lib.rpc_dense_conv(0, _ffi.ptr(x), ci, ci, _ffi.ptr(wt), co, _ffi.ptr(z), co, 0, 0, _ffi.ptr(part),
                                       img, img, img, _ffi.stream_of(z))
                run(); run()
                e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
                e0.record(st)
                for _ in range(iters):
                    run()
                e1.record(st)
                e1.synchronize()
                times[d].append(e0.elapsed_time(e1) * 1e3 / iters)
        lib.rpc_dense_tune(4, 0)
        names = {0: "y_real", 1: "y_no_mfma", 17: "y_no_kloop", 64: "y_no_stores", 65: "y_no_mfma_no_stores", 81: "y_skeleton", 128: "former_loop"}
        print(f"B{B} {H}x{W} {ci}->{co}", json.dumps({names[d]: round(sorted(v)[len(v) // 2], 2) for d, v in times.items()}),
              flush=True)


if __name__ == "__main__":
    main()
