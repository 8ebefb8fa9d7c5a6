"""rpc_head_unpack_grad(_f32): the fp32 head-output gradient slice [cells][dp] at channel offset doff becomes the padded
dz image [cells][zp] (the n real channels cast to the engine's dtype, the padding zero) and dbias = the n column
sums (fixed-order two-level, checked against float64), for the pitches and widths of CenterHead's final convs (zp = 64,
n = 1..10 at 4 x 128 x 128 cells) and odd ones."""
import pytest
import torch

from robustpointclouds_amd import _ffi

DEV = torch.device("cuda")


@pytest.mark.gpu
@pytest.mark.parametrize("f32", [False, True])
@pytest.mark.parametrize("cells,dp,doff,n,zp", [(4 * 128 * 128, 10, 0, 2, 64), (4 * 128 * 128, 60, 10, 10, 64),
                                                 (65535, 16, 0, 16, 64), (1000, 12, 3, 1, 16), (777, 8, 0, 5, 8),
                                                 (5000, 30, 6, 7, 24)])
def test_head_unpack(f32, cells, dp, doff, n, zp):
    lib = _ffi.load()
    g = torch.Generator().manual_seed(cells + n)
    dout = torch.randn(cells, dp, generator=g).to(DEV)
    dt = torch.float32 if f32 else torch.bfloat16
    dz = torch.full((cells, zp), 7.0, dtype=dt, device=DEV)   # the padding must be overwritten with zeros
    db = torch.empty(n, device=DEV)
    wsz = lib.rpc_head_unpack_workspace_size()
    ws = _ffi.workspace(wsz, DEV)
    fn = lib.rpc_head_unpack_grad_f32 if f32 else lib.rpc_head_unpack_grad
    _ffi.check(fn(_ffi.ptr(dout), dp, doff, n, _ffi.ptr(dz), zp, cells, _ffi.ptr(db), _ffi.ptr(ws), wsz,
                  _ffi.stream_of(dz)), "rpc_head_unpack_grad")
    torch.cuda.synchronize()
    want = torch.zeros(cells, zp, dtype=dt, device=DEV)
    want[:, :n] = dout[:, doff:doff + n].to(dt)
    assert torch.equal(dz, want)
    ref = dout[:, doff:doff + n].double().sum(0)
    scale = dout[:, doff:doff + n].double().abs().sum(0)
    assert torch.all((db.double() - ref).abs() <= 1e-5 * scale + 1e-6)
