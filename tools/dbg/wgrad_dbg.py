import torch, torch.nn.functional as F
from robustpointclouds_amd import _ffi
DEV = torch.device("cuda")
lib = _ffi.load()

def run(fmap, kind, x, dz, Wshape, R, S, O, ci, co):
    dW = torch.empty(Wshape, dtype=torch.float32, device=DEV)
    wsz = lib.rpc_dense_wgrad_workspace_size(fmap, _ffi.int_arr(R), ci, co)
    ws = _ffi.workspace(wsz, DEV)
    xn = x.permute(0, 2, 3, 1).contiguous().to(DEV); dn = dz.permute(0, 2, 3, 1).contiguous().to(DEV)
    _ffi.check(lib.rpc_dense_wgrad(fmap, kind, _ffi.ptr(xn), ci, ci, _ffi.ptr(dn), co, co, _ffi.int_arr(R),
               _ffi.int_arr(S), _ffi.int_arr(O), _ffi.ptr(dW), _ffi.ptr(ws), wsz, _ffi.stream_of(dW)), "wg")
    torch.cuda.synchronize()
    return dW.cpu().double()

B, H, W, c = 1, 8, 8, 128
x = torch.ones(B, c, H, W, dtype=torch.bfloat16); dz = torch.ones(B, c, H, W, dtype=torch.bfloat16)
g = run(0, 0, x, dz, (c, c, 3, 3), (B, H, W), (B, H, W), (B, H, W), c, c)
print("ones S1 tap counts (expect 49 56 49 / 56 64 56 / 49 56 49):")
print(g[0, 0]); print("min/max over ci,co per tap", g.amin((0, 1)), g.amax((0, 1)))
# P1 pure gemm
x = torch.randn(B, c, H, W).to(torch.bfloat16); dz = torch.randn(B, 256, H, W).to(torch.bfloat16)
g = run(3, 1, x, dz, (c, 256, 1, 1), (B, H, W), (B, H, W), (B, H, W), c, 256)
want = torch.einsum("bchw,bdhw->cd", x.double(), dz.double())
print("P1 err", (g[:, :, 0, 0] - want).abs().max().item(), want.abs().max().item())
# identity-ish: x one-hot channel 3 at pixel 0, dz one-hot channel 5 at pixel 0
x = torch.zeros(B, c, H, W, dtype=torch.bfloat16); x[0, 3, 0, 0] = 1
dz = torch.zeros(B, 256, H, W, dtype=torch.bfloat16); dz[0, 5, 0, 0] = 1
g = run(3, 1, x, dz, (c, 256, 1, 1), (B, H, W), (B, H, W), (B, H, W), c, 256)
nz = g[:, :, 0, 0].nonzero()
print("one-hot nonzeros", nz.tolist()[:10], g[:, :, 0, 0][g[:, :, 0, 0] != 0].tolist()[:10])
x = torch.zeros(B, c, H, W, dtype=torch.bfloat16); x[0, 3, 2, 5] = 1
dz = torch.zeros(B, 256, H, W, dtype=torch.bfloat16); dz[0, 5, 2, 5] = 1
g = run(3, 1, x, dz, (c, 256, 1, 1), (B, H, W), (B, H, W), (B, H, W), c, 256)
nz = g[:, :, 0, 0].nonzero()
print("one-hot pixel 21 nonzeros", nz.tolist()[:10], g[:, :, 0, 0][g[:, :, 0, 0] != 0].tolist()[:10])
for (B, H, W) in [(1, 16, 16), (2, 24, 20)]:
    x = torch.ones(B, c, H, W, dtype=torch.bfloat16); dz = torch.ones(B, c, H, W, dtype=torch.bfloat16)
    g = run(0, 0, x, dz, (c, c, 3, 3), (B, H, W), (B, H, W), (B, H, W), c, c)
    print(B, H, W, "ones S1 taps min", g.amin((0, 1)).flatten().tolist(), "max", g.amax((0, 1)).flatten().tolist())
    x = torch.randn(B, c, H, W).to(torch.bfloat16); dz = torch.randn(B, 256, H, W).to(torch.bfloat16)
    g = run(3, 1, x, dz, (c, 256, 1, 1), (B, H, W), (B, H, W), (B, H, W), c, 256)
    want = torch.einsum("bchw,bdhw->cd", x.double(), dz.double())
    print("P1 err", (g[:, :, 0, 0] - want).abs().max().item(), want.abs().max().item())
    # rows one-hot: x channel 0 = pixel index (small ints), dz channel 0 = 1 -> sum of pixel ids
    x = torch.zeros(B, c, H, W, dtype=torch.bfloat16); x[:, 0] = 1.0
    dz = torch.zeros(B, 256, H, W, dtype=torch.bfloat16)
    for p in range(B * H * W):
        b, r = divmod(p, H * W); dz[b, p % 256, r // W, r % W] = 1.0
    g = run(3, 1, x, dz, (c, 256, 1, 1), (B, H, W), (B, H, W), (B, H, W), c, 256)
    want = torch.einsum("bchw,bdhw->cd", x.double(), dz.double())
    print("row-count err", (g[:, :, 0, 0] - want).abs().max().item(), g[0, :8, 0, 0].tolist(), want[0, :8].tolist())
