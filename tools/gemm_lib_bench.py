"""Microbenchmark: the P1 (1x1) GEMM shapes of the KITTI 3-class step on the dense engine (rpc_dense_conv
P1 / rpc_dense_wgrad P1) vs torch.matmul (hipBLASLt) on the same bf16 operands. Prints us per call."""
import torch

from robustpointclouds_amd import _ffi

P1 = 3
dev = torch.device("cuda")
lib = _ffi.load()


def timeit(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1000


B, H, W = 6, 200, 176
M = B * H * W
img = _ffi.int_arr((B, H, W))
for ci, co in [(512, 128), (128, 512), (128, 256), (256, 128)]:
    x = torch.randn(M, ci, device=dev).to(torch.bfloat16)
    wt = (torch.randn(co, ci, device=dev) * 0.05).to(torch.bfloat16)     # [co][ci] = the engine's fwd operand
    out = torch.empty(M, co, device=dev, dtype=torch.bfloat16)
    st = _ffi.stream_of(out)
    eng = lambda: lib.rpc_dense_conv(P1, _ffi.ptr(x), ci, ci, _ffi.ptr(wt), co, _ffi.ptr(out), co, 0, 0, None, img,
                                     img, img, st)
    t_eng = timeit(eng)
    ref = out.clone()
    o2 = torch.empty_like(out)
    lib_fn = lambda: torch.matmul(x, wt.t(), out=o2)
    t_lib = timeit(lib_fn)
    err = (o2.float() - ref.float()).abs().max().item()
    # weight gradient dW[co][ci] = dz^T x (fp32 result)
    dz = torch.randn(M, co, device=dev).to(torch.bfloat16)
    wsz = lib.rpc_dense_wgrad_workspace_size(P1, img, ci, co)
    ws = _ffi.workspace(wsz, dev)
    dW = torch.empty(ci, co, 1, 1, device=dev)
    eng_w = lambda: lib.rpc_dense_wgrad(P1, 1, _ffi.ptr(x), ci, ci, _ffi.ptr(dz), co, co, img, img, img, _ffi.ptr(dW),
                                        _ffi.ptr(ws), wsz, st)
    t_eng_w = timeit(eng_w)
    dW2 = torch.empty(co, ci, device=dev, dtype=torch.bfloat16)
    lib_w = lambda: torch.matmul(dz.t(), x, out=dW2)
    t_lib_w = timeit(lib_w)
    dW3 = torch.empty(co, ci, device=dev, dtype=torch.float32)
    lib_w32 = lambda: torch.mm(dz.t(), x, out_dtype=torch.float32, out=dW3) if hasattr(torch.mm, "__call__") else None
    try:
        t_lib_w32 = timeit(lib_w32)
    except Exception as e:  # noqa: BLE001
        t_lib_w32 = float("nan")
    print(f"{ci:4d}->{co:4d}  fwd engine {t_eng:7.1f} us  torch.matmul {t_lib:7.1f} us (max diff {err:.3g})  "
          f"wgrad engine {t_eng_w:7.1f} us  torch bf16-out {t_lib_w:7.1f} us  fp32-out {t_lib_w32:7.1f} us", flush=True)
