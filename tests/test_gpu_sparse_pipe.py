"""The sparse 16-bit GEMM's BatchNorm finalize fused into the data-gradient launches (rpc_spconv_gemm_bf16_fin)
against the separate finalize, on random maps and on the real SECOND rulebooks of a synthetic KITTI batch (whole
bf16 SparseEncoder forward + backward), and the basicblock residual backward (alone, at every width, and fused
into the data-gradient epilogue). (r05's per-block source-row union path, bit-identical but slower, was removed:
profiles/r05_union_ab.txt.)"""
import pytest
import torch

from robustpointclouds_amd import _ffi

pytestmark = pytest.mark.gpu


def _r8(c):
    return (c + 7) // 8 * 8


def _run(lib, a, n_src, kg, nbr, K, rev, n_out, bt, ng, epi, ez, ebn, dev):
    out = torch.full((n_out, ng), float("nan"), device=dev)
    nblk = max(lib.rpc_spconv_gemm_blocks(n_out), 1)
    part = torch.full((nblk, 2 * ng), float("nan"), device=dev) if epi != 2 else None
    _ffi.check(lib.rpc_spconv_gemm_h16(_ffi.ptr(a), 0, n_src, kg, _ffi.ptr(nbr), K, rev, n_out, _ffi.ptr(bt), ng,
                                       _ffi.ptr(out), _ffi.ptr(ez), _ffi.ptr(ebn), _ffi.ptr(part), epi,
                                       _ffi.stream_of(out)), "rpc_spconv_gemm_h16")
    torch.cuda.synchronize()
    return out, part


def _encoder_case():
    from robustpointclouds_amd import voxelize
    from robustpointclouds_amd.sparse_encoder import SparseEncoder
    from robustpointclouds_amd.synthetic import KITTI_PC_RANGE, KITTI_VOXEL_SIZE, kitti_batch
    dev = torch.device("cuda")
    pts, _, _ = kitti_batch(6, seed0=0, num_classes=3)
    pts = [torch.from_numpy(p).to(dev) for p in pts]
    d = voxelize.Voxelization(KITTI_VOXEL_SIZE, KITTI_PC_RANGE, 5, 16000).to(dev).voxelize_frames(pts)
    feats = (d["voxels"][:, :, :4].sum(1) / d["num_points"].clamp(min=1).view(-1, 1).float()).contiguous()
    torch.manual_seed(0)
    enc = SparseEncoder(4, [41, 1600, 1408]).to(dev)
    enc.bf16 = enc.dense_nhwc = enc.dense_bf16 = True
    return enc, feats, d["coors"]


def _encoder_step(enc, feats, coors, fused, fmt=1):
    from robustpointclouds_amd import sparse_encoder as se
    prev_f, prev_fmt = se.FUSED_FINALIZE, se.FWD_FMT
    se.FUSED_FINALIZE, se.FWD_FMT = fused, fmt
    try:
        for p in enc.parameters():
            p.grad = None
        bns = [m[1] for m in enc.layers()]
        saved = [(b.running_mean.clone(), b.running_var.clone()) for b in bns]
        f = feats.clone().requires_grad_(True)
        out = enc(f, coors, 6)
        g = torch.Generator(device="cpu").manual_seed(1)
        out.backward(torch.randn(out.shape, generator=g).to(out.device).to(out.dtype))
        torch.cuda.synchronize()
        stats = [torch.cat([b.running_mean, b.running_var]).clone() for b in bns]
        for b, (m, v) in zip(bns, saved):   # every run starts from the same running statistics
            b.running_mean.copy_(m)
            b.running_var.copy_(v)
        return out.detach().float().clone(), f.grad.clone(), [p.grad.clone() for p in enc.parameters()], stats
    finally:
        se.FUSED_FINALIZE, se.FWD_FMT = prev_f, prev_fmt


def test_fused_finalize_matches_separate_and_is_deterministic():
    """BatchNorm-backward finalizes fused into the data-gradient GEMMs (two-level last-block sums) against the
    separate rpc_bn_finalize launches: bit-identical from run to run, the ticket counters back at zero after every
    launch, and the same results up to the double-sum order of the statistics, whose last-bit differences could
    flip a bf16 rounding or a ReLU mask downstream (relative L2 <= 5e-2 on the BEV, every gradient and the running
    statistics; measured 0: bit-identical on this case, r04)."""
    enc, feats, coors = _encoder_case()
    ref = _encoder_step(enc, feats, coors, False)
    a = _encoder_step(enc, feats, coors, True)
    b = _encoder_step(enc, feats, coors, True)
    for x, y in zip([a[0], a[1]] + a[2] + a[3], [b[0], b[1]] + b[2] + b[3]):
        assert torch.equal(x, y)
    worst = 0.0
    for i, (x, y) in enumerate(zip([ref[0], ref[1]] + ref[2] + ref[3], [a[0], a[1]] + a[2] + a[3])):
        d = ((x.double() - y.double()).norm() / max(y.double().norm().item(), 1e-30)).item()
        worst = max(worst, d)
        assert d < 5e-2, (i, d)
    print(f"fused vs separate finalize: worst relative L2 {worst:.2e}")
    assert int(enc.fin_tickets(feats.device).abs().sum().item()) == 0


@pytest.mark.parametrize("kg,ng,n_out", [(64, 64, 106000), (32, 64, 5000), (64, 128, 130), (128, 128, 64),
                                         (16, 32, 1)])
def test_gemm_fin_entry_point(kg, ng, n_out):
    """rpc_spconv_gemm_bf16_fin alone (data gradient, epi 1): the same output rows as the unfused GEMM, the
    finalize outputs of rpc_bn_finalize mode 1 on the same partial rows (bnb, dgamma, dbeta) to
    double-summation-order accuracy, repeated launches reuse the re-armed tickets."""
    lib = _ffi.load()
    dev = torch.device("cuda")
    g = torch.Generator().manual_seed(n_out + kg)
    K, n_src = 27, max(n_out, 1000)
    nbr = torch.randint(0, n_src, (n_out, K), generator=g, dtype=torch.int32)
    nbr[torch.rand((n_out, K), generator=g) > 0.3] = -1
    a = torch.zeros((n_src, _r8(kg)), dtype=torch.bfloat16)
    a[:, :kg] = torch.randn((n_src, kg), generator=g).to(torch.bfloat16)
    W = torch.randn((K, kg, ng), generator=g) * 0.1
    a, nbr, W = a.to(dev), nbr.to(dev), W.to(dev)
    bt = torch.empty(lib.rpc_spconv_bf16_weight_elems(K, kg, ng, 0), dtype=torch.bfloat16, device=dev)
    _ffi.check(lib.rpc_spconv_prep_weight_bf16(_ffi.ptr(W), K, kg, ng, 0, _ffi.ptr(bt), _ffi.stream_of(bt)), "prep")
    ez = torch.randn((n_out, ng), generator=g).to(dev)
    ebn = torch.cat([torch.rand(ng, generator=g) + 0.5, torch.randn(ng, generator=g) * 0.1,
                     torch.randn(ng, generator=g) * 0.1, torch.rand(ng, generator=g) + 0.5]).to(dev)
    gamma, beta = (torch.rand(ng, generator=g) + 0.5).to(dev), torch.randn(ng, generator=g).to(dev)
    ticket = torch.zeros(lib.rpc_bn_fin_tickets(n_out), dtype=torch.int32, device=dev)
    gpart = torch.empty(lib.rpc_bn_fin_groups(n_out) * 2 * ng, dtype=torch.float64, device=dev)
    nblk = lib.rpc_spconv_gemm_blocks(n_out)
    st = _ffi.stream_of(ez)
    for rep in range(3):
        out = torch.full((n_out, ng), float("nan"), device=dev)
        part = torch.full((nblk, 2 * ng), float("nan"), device=dev)
        bn = torch.full((5 * ng,), float("nan"), device=dev)
        dg, db = torch.full((ng,), float("nan"), device=dev), torch.full((ng,), float("nan"), device=dev)
        fin = _ffi.RpcBnFin(ticket.data_ptr(), gpart.data_ptr(), 1, gamma.data_ptr(), beta.data_ptr(), 1e-3, 0.01,
                            None, None, ebn.data_ptr(), bn.data_ptr(), dg.data_ptr(), db.data_ptr())
        _ffi.check(lib.rpc_spconv_gemm_bf16_fin(_ffi.ptr(a), n_src, kg, _ffi.ptr(nbr), K, 0, n_out, _ffi.ptr(bt), ng,
                                                _ffi.ptr(out), _ffi.ptr(ez), _ffi.ptr(ebn), _ffi.ptr(part), 1,
                                                _ffi.C.byref(fin), st), "rpc_spconv_gemm_bf16_fin")
        ref_out, ref_part = _run(lib, a, n_src, kg, nbr, K, 0, n_out, bt, ng, 1, ez, ebn, dev)
        assert torch.equal(out, ref_out)
        assert torch.equal(part, ref_part)
        rbn = torch.full((5 * ng,), float("nan"), device=dev)
        rdg, rdb = torch.full((ng,), float("nan"), device=dev), torch.full((ng,), float("nan"), device=dev)
        _ffi.check(lib.rpc_bn_finalize(_ffi.ptr(part), nblk, ng, n_out, 1, _ffi.ptr(gamma), _ffi.ptr(beta), 1e-3,
                                       0.01, None, None, _ffi.ptr(ebn), _ffi.ptr(rbn), _ffi.ptr(rdg), _ffi.ptr(rdb),
                                       None, st), "rpc_bn_finalize")
        torch.cuda.synchronize()
        for x, y in [(bn, rbn), (dg, rdg), (db, rdb)]:
            assert torch.isfinite(x).all()
            assert torch.allclose(x, y, rtol=1e-6, atol=1e-6 * max(y.abs().max().item(), 1.0))
        assert int(ticket.abs().sum().item()) == 0


@pytest.mark.parametrize("kg,ng,n_out,K,g2", [(32, 32, 3000, 27, True), (128, 128, 700, 27, False),
                                               (64, 64, 129, 3, True), (16, 16, 1, 27, True)])
def test_gemm_res_matches_separate_residual_backward(kg, ng, n_out, K, g2):
    """rpc_spconv_gemm_res (the basicblock residual backward in the data-gradient epilogue) against the plain
    GEMM followed by rpc_sparse_res_backward: m = (dgrad + g2) * [out > 0] bit-identical, the BatchNorm-backward
    partial rows equal up to the summation order (the same 64-row groups)."""
    lib = _ffi.load()
    dev = torch.device("cuda")
    g = torch.Generator().manual_seed(n_out + kg + K)
    n_src = max(n_out, 500)
    nbr = torch.randint(0, n_src, (n_out, K), generator=g, dtype=torch.int32)
    nbr[torch.rand((n_out, K), generator=g) > 0.3] = -1
    a = torch.zeros((n_src, _r8(kg)), dtype=torch.bfloat16)
    a[:, :kg] = torch.randn((n_src, kg), generator=g).to(torch.bfloat16)
    W = torch.randn((K, kg, ng), generator=g) * 0.1
    a, nbr, W = a.to(dev), nbr.to(dev), W.to(dev)
    st = _ffi.stream_of(W)
    bt = torch.empty(lib.rpc_spconv_bf16_weight_elems(K, kg, ng, 0), dtype=torch.bfloat16, device=dev)
    _ffi.check(lib.rpc_spconv_prep_weight_bf16(_ffi.ptr(W), K, kg, ng, 0, _ffi.ptr(bt), st), "prep")
    out = torch.randn((n_out, ng), generator=g).to(dev)
    z = torch.randn((n_out, ng), generator=g).to(dev)
    gid = torch.randn((n_out, ng), generator=g).to(dev) if g2 else None
    bn = torch.cat([torch.rand(ng, generator=g) + 0.5, torch.randn(ng, generator=g) * 0.1,
                    torch.randn(ng, generator=g) * 0.1, torch.rand(ng, generator=g) + 0.5]).to(dev)
    nblk = max(lib.rpc_spconv_gemm_blocks(n_out), 1)
    # separate: plain GEMM, then the residual pass
    din, _ = _run(lib, a, n_src, kg, nbr, K, 0, n_out, bt, ng, 2, None, None, dev)
    m_ref = torch.full((n_out, ng), float("nan"), device=dev)
    p_ref = torch.full((nblk, 2 * ng), float("nan"), device=dev)
    _ffi.check(lib.rpc_sparse_res_backward(_ffi.ptr(gid) if g2 else _ffi.ptr(din), _ffi.ptr(din) if g2 else None,
                                           _ffi.ptr(out), _ffi.ptr(z), _ffi.ptr(bn), n_out, ng, _ffi.ptr(m_ref),
                                           _ffi.ptr(p_ref), st), "rpc_sparse_res_backward")
    # fused
    m = torch.full((n_out, ng), float("nan"), device=dev)
    p = torch.full((nblk, 2 * ng), float("nan"), device=dev)
    _ffi.check(lib.rpc_spconv_gemm_res(_ffi.ptr(a), n_src, kg, _ffi.ptr(nbr), K, 0, n_out, _ffi.ptr(bt), ng,
                                       _ffi.ptr(m), _ffi.ptr(gid) if g2 else None, _ffi.ptr(out), _ffi.ptr(z),
                                       _ffi.ptr(bn), _ffi.ptr(p), None, st), "rpc_spconv_gemm_res")
    torch.cuda.synchronize()
    assert torch.equal(m, m_ref)
    scale = torch.cat([m.abs().sum(0), (m * ((z - bn[2 * ng:3 * ng]) * bn[3 * ng:])).abs().sum(0)])
    assert torch.all((p.sum(0) - p_ref.sum(0)).abs() <= 1e-5 * scale + 1e-6)


@pytest.mark.parametrize("c", [16, 48, 64, 96, 128, 200])
@pytest.mark.parametrize("n", [1, 333, 4100])
def test_res_backward_any_width(c, n):
    """rpc_sparse_res_backward at every width, including the ones whose c / 4 is not a power of two (those take
    the per-element kernel; the vectorized one tiles a wave with c / 4 lanes): m = (g1 + g2) * [out > 0] exact,
    the (sum m, sum m * xhat) rows of every 64-row group against torch in float64."""
    lib = _ffi.load()
    dev = torch.device("cuda")
    g = torch.Generator().manual_seed(c * 7 + n)
    g1, g2, out, z = (torch.randn((n, c), generator=g).to(dev) for _ in range(4))
    bn = torch.cat([torch.rand(c, generator=g) + 0.5, torch.randn(c, generator=g) * 0.1,
                    torch.randn(c, generator=g) * 0.1, torch.rand(c, generator=g) + 0.5]).to(dev)
    ngr = lib.rpc_spconv_gemm_blocks(n)
    m = torch.full((n, c), float("nan"), device=dev)
    part = torch.full((ngr + 1, 2 * c), float("nan"), device=dev)   # one guard row past the groups
    _ffi.check(lib.rpc_sparse_res_backward(_ffi.ptr(g1), _ffi.ptr(g2), _ffi.ptr(out), _ffi.ptr(z), _ffi.ptr(bn), n, c,
                                           _ffi.ptr(m), _ffi.ptr(part), _ffi.stream_of(m)), "rpc_sparse_res_backward")
    torch.cuda.synchronize()
    m_ref = (g1 + g2) * (out > 0)
    assert torch.equal(m, m_ref)
    xh = (z.double() - bn[2 * c:3 * c].double()) * bn[3 * c:].double()
    pad = ngr * 64 - n
    md = torch.cat([m_ref.double(), torch.zeros((pad, c), dtype=torch.float64, device=dev)]).view(ngr, 64, c)
    xd = torch.cat([xh, torch.zeros((pad, c), dtype=torch.float64, device=dev)]).view(ngr, 64, c)
    s1, s2 = md.sum(1), (md * xd).sum(1)
    scale1, scale2 = md.abs().sum(1), (md * xd).abs().sum(1)
    assert torch.all((part[:ngr, :c].double() - s1).abs() <= 1e-5 * scale1 + 1e-6)
    assert torch.all((part[:ngr, c:].double() - s2).abs() <= 1e-5 * scale2 + 1e-6)
    assert torch.isnan(part[ngr]).all()     # nothing written past the last group
