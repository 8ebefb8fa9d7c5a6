"""Micro-benchmark of the DCN kernels at the CenterPoint nuScenes head size (B=4, 128 x 128)."""
import sys
import os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from robustpointclouds_amd import _ffi
from robustpointclouds_amd import dense_bev as db

B, H, W = 4, 128, 128
amp = float(sys.argv[1]) if len(sys.argv) > 1 else 0.0
dev = torch.device("cuda")
lib = _ffi.load()
st = _ffi.stream_of(torch.empty(1, device=dev))
g = torch.Generator(device="cpu").manual_seed(0)
x = db._nhwc(torch.randn(B, 64, H, W, generator=g).to(dev))
oz = db._nhwc((torch.randn(B, 64, H, W, generator=g) * amp).to(dev))
ob = torch.zeros(18, device=dev)
W32 = (torch.randn(64, 16, 3, 3, generator=g) * 0.1).to(dev)
wf = torch.empty((9, 64, 64), dtype=torch.bfloat16, device=dev)
wd = torch.empty((9, 64, 64), dtype=torch.bfloat16, device=dev)
lib.rpc_dcn_prep_weight(_ffi.ptr(W32), _ffi.ptr(wf), _ffi.ptr(wd), st)
out = db._image(B, 64, H, W, dev)
gi = db._nhwc(torch.randn(B, 64, H, W, generator=g).to(dev))
dx = torch.zeros((B * H * W, 64), device=dev)
doff = db._image(B, 64, H, W, dev)
dob = torch.empty(18, device=dev)
dW = torch.empty((64, 16, 3, 3), device=dev)
wsz = lib.rpc_dcn_backward_workspace_size(B, H, W)
ws = torch.empty(wsz, dtype=torch.uint8, device=dev)
for name, fn in (("fwd", lambda: lib.rpc_dcn_forward(_ffi.ptr(x), 64, _ffi.ptr(oz), 64, _ffi.ptr(ob), _ffi.ptr(wf),
                                                     _ffi.ptr(out), 64, B, H, W, st)),
                 ("bwd", lambda: lib.rpc_dcn_backward(_ffi.ptr(x), 64, _ffi.ptr(oz), 64, _ffi.ptr(ob), _ffi.ptr(wd),
                                                      _ffi.ptr(gi), 64, _ffi.ptr(dx), _ffi.ptr(doff), 64, _ffi.ptr(dob),
                                                      _ffi.ptr(dW), B, H, W, _ffi.ptr(ws), wsz, st))):
    for _ in range(3):
        assert fn() == 0
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        fn()
    e1.record()
    torch.cuda.synchronize()
    print(f"{name} amp={amp}: {e0.elapsed_time(e1) / 10 * 1000:.1f} us/call", flush=True)
