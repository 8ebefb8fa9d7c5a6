"""bf16 sparse-conv kernels in isolation: with bf16 operands fixed, the MFMA kernels must match
a float64 matmul of the same (exactly representable) bf16 values to fp32-accumulation accuracy.
Covers every (C_in, C_out) pair SECOND's SparseEncoder uses, ragged row counts (not multiples of
the 32/64-row tiles), empty offsets and rows with no neighbour at all."""
import numpy as np
import pytest
import torch

from robustpointclouds_amd import _ffi

pytestmark = pytest.mark.gpu

PAIRS = [(16, 16), (16, 32), (32, 32), (32, 64), (64, 64), (64, 128), (128, 128)]


def _r8(c):
    return (c + 7) // 8 * 8


def _case(n_out, n_in, K, ci, co, density, seed):
    g = torch.Generator().manual_seed(seed)
    nbr = torch.randint(0, n_in, (n_out, K), generator=g, dtype=torch.int32)
    nbr[torch.rand((n_out, K), generator=g) > density] = -1
    if K > 2:
        nbr[:, 1] = -1          # an offset nobody uses
    h = torch.zeros((n_in, _r8(ci)), dtype=torch.bfloat16)
    h[:, :ci] = torch.randn((n_in, ci), generator=g).to(torch.bfloat16)
    dz = torch.zeros((n_out, _r8(co)), dtype=torch.bfloat16)
    dz[:, :co] = torch.randn((n_out, co), generator=g).to(torch.bfloat16)
    return nbr, h, dz


def _wgrad_ref(nbr, h, dz, K, ci, co):
    dW = torch.zeros((K, ci, co), dtype=torch.float64)
    hd, dd = h[:, :ci].double(), dz[:, :co].double()
    for k in range(K):
        ok = nbr[:, k] >= 0
        if ok.any():
            dW[k] = hd[nbr[ok, k].long()].T @ dd[ok]
    return dW


@pytest.mark.parametrize("ci,co", PAIRS)
@pytest.mark.parametrize("n_out,K", [(5000, 27), (1, 27), (3001, 3)])
def test_wgrad_bf16_matches_fp64(ci, co, n_out, K):
    lib = _ffi.load()
    dev = torch.device("cuda")
    nbr, h, dz = _case(n_out, 4000, K, ci, co, 0.3, seed=ci * 1000 + co + n_out)
    ref = _wgrad_ref(nbr, h, dz, K, ci, co)
    dW = torch.full((K, ci, co), float("nan"), device=dev)
    wsz = lib.rpc_spconv_wgrad_bf16_workspace_size(n_out, K, ci, co)
    ws = _ffi.workspace(wsz, dev)
    hd, nd, dd = h.to(dev), nbr.to(dev), dz.to(dev)
    _ffi.check(lib.rpc_spconv_wgrad_bf16(_ffi.ptr(hd), ci, _ffi.ptr(nd), K, n_out, _ffi.ptr(dd), co, _ffi.ptr(dW),
                                         _ffi.ptr(ws), wsz, _ffi.stream_of(dW)), "wgrad_bf16")
    got = dW.cpu().double()
    assert torch.isfinite(got).all()
    # fp32 accumulation of exact bf16 products: relative error ~1e-6 of the row-sum magnitude
    tol = 1e-5 * max(ref.abs().max().item(), 1.0) + 1e-6 * (n_out ** 0.5)
    assert (got - ref).abs().max().item() <= tol
    assert got[1].abs().max().item() == 0.0 if K > 2 else True
    # fixed-order reduction: bitwise deterministic
    dW2 = torch.empty_like(dW)
    _ffi.check(lib.rpc_spconv_wgrad_bf16(_ffi.ptr(hd), ci, _ffi.ptr(nd), K, n_out, _ffi.ptr(dd), co, _ffi.ptr(dW2),
                                         _ffi.ptr(ws), wsz, _ffi.stream_of(dW)), "wgrad_bf16")
    assert torch.equal(dW, dW2)


def test_wgrad_bf16_rejects_short_workspace_and_empty():
    lib = _ffi.load()
    dev = torch.device("cuda")
    nbr, h, dz = _case(100, 50, 27, 16, 16, 0.5, 0)
    dW = torch.full((27, 16, 16), 1.0, device=dev)
    wsz = lib.rpc_spconv_wgrad_bf16_workspace_size(100, 27, 16, 16)
    ws = _ffi.workspace(wsz, dev)
    hd, nd, dd = h.to(dev), nbr.to(dev), dz.to(dev)
    st = _ffi.stream_of(dW)
    assert lib.rpc_spconv_wgrad_bf16(_ffi.ptr(hd), 16, _ffi.ptr(nd), 27, 100, _ffi.ptr(dd), 16, _ffi.ptr(dW),
                                     _ffi.ptr(ws), wsz - 4, st) == 2   # RPC_ERR_WORKSPACE
    assert lib.rpc_spconv_wgrad_bf16(_ffi.ptr(hd), 16, _ffi.ptr(nd), 27, 100, _ffi.ptr(dd), 24, _ffi.ptr(dW),
                                     _ffi.ptr(ws), wsz, st) == 3       # RPC_ERR_UNSUPPORTED
    _ffi.check(lib.rpc_spconv_wgrad_bf16(_ffi.ptr(hd), 16, _ffi.ptr(nd), 27, 0, _ffi.ptr(dd), 16, _ffi.ptr(dW),
                                         _ffi.ptr(ws), wsz, st), "wgrad_bf16(empty)")
    assert dW.abs().max().item() == 0.0


def _bf16_ulp_close(got, want, atol=1e-30):
    """got (bf16 on the GPU) within one bf16 ulp of the float64 value want (+ atol: the fp32 rounding of
    the kernel's intermediate terms where they cancel)."""
    g = got.float().double().cpu()
    w = want.double()
    ulp = w.abs() * 2.0 ** -7
    assert ((g - w).abs() <= ulp + atol).all(), float(((g - w).abs() - ulp).max())


@pytest.mark.parametrize("n,c", [(4097, 64), (333, 16), (1000, 128), (515, 60), (600001, 64), (70001, 128)])
def test_bf16_row_producers(n, c):
    """rpc_to_bf16_rows (relu(bn(z)) -> bf16 rows of pitch round8(C)) and rpc_bnbwd_to_bf16_rows
    (gi * (dy - m1 - xhat*m2) -> bf16): the 8-channel vector forms (C % 8 == 0) and the scalar form
    (C = 60, padded channels zero) against float64 within one bf16 ulp."""
    lib = _ffi.load()
    dev = torch.device("cuda")
    g = torch.Generator().manual_seed(n + c)
    cp = _r8(c)
    z = torch.randn(n, c, generator=g) * 2
    dy = torch.randn(n, c, generator=g)
    bn = torch.cat([torch.rand(c, generator=g) + 0.5, torch.randn(c, generator=g) * 0.3,
                    torch.randn(c, generator=g) * 0.2, torch.rand(c, generator=g) + 0.5])
    bnb = torch.cat([torch.rand(c, generator=g) + 0.5] + [torch.randn(c, generator=g) * 0.3 for _ in range(4)])
    zd, dyd, bnd, bnbd = z.to(dev), dy.to(dev), bn.to(dev), bnb.to(dev)
    h = torch.full((n, cp), 7.0, dtype=torch.bfloat16, device=dev)
    dz = torch.full((n, cp), 7.0, dtype=torch.bfloat16, device=dev)
    st = _ffi.stream_of(h)
    _ffi.check(lib.rpc_to_bf16_rows(_ffi.ptr(zd), _ffi.ptr(bnd), n, c, 1, _ffi.ptr(h), st), "rpc_to_bf16_rows")
    _ffi.check(lib.rpc_bnbwd_to_bf16_rows(_ffi.ptr(dyd), _ffi.ptr(zd), _ffi.ptr(bnbd), n, c, _ffi.ptr(dz), st),
               "rpc_bnbwd_to_bf16_rows")
    torch.cuda.synchronize()
    sc, be, mu = bn.double().view(4, c)[:3]
    want_h = torch.clamp((z.double() - mu) * sc + be, min=0.0)
    gi, m1, m2, mb, ib = bnb.double().view(5, c)
    want_dz = gi * (dy.double() - m1 - (z.double() - mb) * ib * m2)
    _bf16_ulp_close(h[:, :c], want_h, atol=1e-6)   # relu(x) with x within fp32 rounding of 0
    _bf16_ulp_close(dz[:, :c], want_dz, atol=1e-5)
    if cp > c:
        assert (h[:, c:] == 0).all() and (dz[:, c:] == 0).all()


@pytest.mark.parametrize("n,c", [(4097, 64), (515, 60), (70001, 128)])
def test_f16_row_producer(n, c):
    """rpc_to_h16_rows fmt 1 (the perf mode's fp16 forward rows): relu(bn(z)) within one fp16 ulp of float64, and
    its bf16 copy within one bf16 ulp."""
    lib = _ffi.load()
    dev = torch.device("cuda")
    g = torch.Generator().manual_seed(n + 7 * c)
    cp = _r8(c)
    z = torch.randn(n, c, generator=g) * 2
    bn = torch.cat([torch.rand(c, generator=g) + 0.5, torch.randn(c, generator=g) * 0.3,
                    torch.randn(c, generator=g) * 0.2, torch.rand(c, generator=g) + 0.5])
    h = torch.full((n, cp), 7.0, dtype=torch.float16, device=dev)
    hb = torch.full((n, cp), 7.0, dtype=torch.bfloat16, device=dev)
    zd, bnd = z.to(dev), bn.to(dev)     # held: the kernel reads them after the call returns
    _ffi.check(lib.rpc_to_h16_rows(_ffi.ptr(zd), _ffi.ptr(bnd), n, c, 1, 1, _ffi.ptr(h), _ffi.ptr(hb),
                                   _ffi.stream_of(h)), "rpc_to_h16_rows")
    torch.cuda.synchronize()
    sc, be, mu = bn.double().view(4, c)[:3]
    want = torch.clamp((z.double() - mu) * sc + be, min=0.0)
    got = h[:, :c].double().cpu()
    assert ((got - want).abs() <= want.abs() * 2.0 ** -10 + 1e-6).all()
    _bf16_ulp_close(hb[:, :c], want, atol=1e-6)      # the bf16 copy of the same rows (weight gradient operand)
    if cp > c:
        assert (h[:, c:] == 0).all() and (hb[:, c:] == 0).all()


@pytest.mark.parametrize("ci,co", [(16, 32), (32, 32), (64, 64), (64, 128), (128, 128)])
def test_gemm_f16_forward_matches_fp64(ci, co):
    """rpc_spconv_gemm_h16 fmt 1 (fp16 rows and fp16 forward weight tiles on v_mfma_f32_16x16x32_f16): against a
    float64 gather-matmul of the same fp16 values, to fp32-accumulation accuracy; the BatchNorm partial rows
    are the column sums of the stored rows; other epilogues refuse fp16."""
    lib = _ffi.load()
    dev = torch.device("cuda")
    n_out, n_in, K = 3001, 2500, 27
    g = torch.Generator().manual_seed(ci * 3 + co)
    nbr = torch.randint(0, n_in, (n_out, K), generator=g, dtype=torch.int32)
    nbr[torch.rand((n_out, K), generator=g) > 0.3] = -1
    h = torch.zeros((n_in, _r8(ci)), dtype=torch.float16)
    h[:, :ci] = (torch.randn((n_in, ci), generator=g) * 3).to(torch.float16)
    W = torch.randn((K, ci, co), generator=g) * 0.05
    hd, nd, Wd = h.to(dev), nbr.to(dev), W.to(dev)
    bt = torch.empty(lib.rpc_spconv_bf16_weight_elems(K, ci, co, 0), dtype=torch.float16, device=dev)
    desc = (_ffi.RpcSpconvWprep * 1)(_ffi.RpcSpconvWprep(Wd.data_ptr(), bt.data_ptr(), K, ci, co, 0, 1))
    st = _ffi.stream_of(Wd)
    _ffi.check(lib.rpc_spconv_prep_weight_bf16_batch(desc, 1, st), "prep fp16")
    out = torch.full((n_out, co), float("nan"), device=dev)
    part = torch.full((lib.rpc_spconv_gemm_blocks(n_out), 2 * co), float("nan"), device=dev)
    _ffi.check(lib.rpc_spconv_gemm_h16(_ffi.ptr(hd), 1, n_in, ci, _ffi.ptr(nd), K, 0, n_out, _ffi.ptr(bt), co,
                                       _ffi.ptr(out), None, None, _ffi.ptr(part), 0, st), "gemm_h16")
    assert lib.rpc_spconv_gemm_h16(_ffi.ptr(hd), 1, n_in, ci, _ffi.ptr(nd), K, 0, n_out, _ffi.ptr(bt), co,
                                   _ffi.ptr(out), None, None, None, 2, st) == 3      # fp16: forward only
    torch.cuda.synchronize()
    Wq = W.to(torch.float16).double()
    ref = torch.zeros((n_out, co), dtype=torch.float64)
    hq = h[:, :ci].double()
    for k in range(K):
        ok = nbr[:, k] >= 0
        ref[ok] += hq[nbr[ok, k].long()] @ Wq[k]
    got = out.double().cpu()
    assert (got - ref).abs().max().item() <= 2e-5 * max(ref.abs().max().item(), 1.0)
    s = part.double().cpu().sum(0)
    assert torch.allclose(s[:co], got.sum(0), rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("ci,co", [(16, 32), (64, 64), (128, 128)])
def test_wgrad_h16_fp16_rows(ci, co):
    """rpc_spconv_wgrad_h16 hfmt 1: the fp16 forward rows are rounded to bf16 as they are staged — the same
    dW as rpc_spconv_wgrad_bf16 on those rows pre-rounded to bf16 (bit for bit)."""
    lib = _ffi.load()
    dev = torch.device("cuda")
    n_out, K = 4000, 27
    nbr, hb, dz = _case(n_out, 3500, K, ci, co, 0.3, seed=ci + co)
    h16 = (hb.float() * 1.37).to(torch.float16)          # values off the bf16 grid
    hq = h16.float().to(torch.bfloat16)                  # what the kernel stages
    wsz = lib.rpc_spconv_wgrad_bf16_workspace_size(n_out, K, ci, co)
    ws = _ffi.workspace(wsz, dev)
    nd, dd = nbr.to(dev), dz.to(dev)
    dW16, dWb = torch.empty((K, ci, co), device=dev), torch.empty((K, ci, co), device=dev)
    st = _ffi.stream_of(dd)
    h16d, hqd = h16.to(dev), hq.to(dev)
    _ffi.check(lib.rpc_spconv_wgrad_h16(_ffi.ptr(h16d), 1, ci, _ffi.ptr(nd), K, n_out, _ffi.ptr(dd), co,
                                        _ffi.ptr(dW16), _ffi.ptr(ws), wsz, st), "wgrad_h16")
    _ffi.check(lib.rpc_spconv_wgrad_bf16(_ffi.ptr(hqd), ci, _ffi.ptr(nd), K, n_out, _ffi.ptr(dd), co,
                                         _ffi.ptr(dWb), _ffi.ptr(ws), wsz, st), "wgrad_bf16")
    torch.cuda.synchronize()
    assert torch.equal(dW16, dWb)


@pytest.mark.parametrize("ci,co,n_out,K,density", [(64, 64, 30001, 27, 0.1), (128, 128, 20000, 27, 0.25),
                                                   (16, 16, 70000, 27, 0.05), (32, 32, 1000, 27, 0.0),
                                                   (64, 128, 513, 3, 1.0)])
def test_wgrad_maps_matches_fp64(ci, co, n_out, K, density):
    """rpc_spconv_wgrad_bf16 on sparse and dense maps, a map with no neighbour at all (density 0), tails of the
    512-row segments and 64-row sub-tiles; fp64 reference on the same bf16 values; deterministic. (r04's pair-list
    variant of this kernel measured slower on the step and was removed in r05.)"""
    lib = _ffi.load()
    dev = torch.device("cuda")
    nbr, h, dz = _case(n_out, 20000, K, ci, co, density, seed=7 + ci + n_out)
    ref = _wgrad_ref(nbr, h, dz, K, ci, co)
    wsz = lib.rpc_spconv_wgrad_bf16_workspace_size(n_out, K, ci, co)
    ws = _ffi.workspace(wsz, dev)
    hd, nd, dd = h.to(dev), nbr.to(dev), dz.to(dev)
    outs = []
    for _ in range(2):
        dW = torch.full((K, ci, co), float("nan"), device=dev)
        _ffi.check(lib.rpc_spconv_wgrad_bf16(_ffi.ptr(hd), ci, _ffi.ptr(nd), K, n_out, _ffi.ptr(dd), co,
                                             _ffi.ptr(dW), _ffi.ptr(ws), wsz, _ffi.stream_of(dW)), "wgrad_bf16")
        outs.append(dW)
    got = outs[0].cpu().double()
    assert torch.isfinite(got).all()
    tol = 1e-5 * max(ref.abs().max().item(), 1.0) + 1e-6 * (n_out ** 0.5)
    assert (got - ref).abs().max().item() <= tol
    assert torch.equal(outs[0], outs[1])
