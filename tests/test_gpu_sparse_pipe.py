"""The LDS-DMA ring sparse GEMM (csrc/spconv_bf16.hip k_gemm_pipe, rpc_spconv_gemm_bf16_mode 1-3) against the
one-offset-look-ahead kernel it replaces (mode 0): the same MFMAs in the same order per accumulator, so
outputs and BatchNorm partial rows must be BIT-identical — for every (GEMM K, output width) instantiation,
the three epilogues, ragged row counts (1, 15, 17, 129 rows: partial waves and blocks), offsets nobody
uses, blocks whose rows have no neighbour at all, and the real SECOND rulebooks of a synthetic KITTI batch
(whole bf16 SparseEncoder forward + backward, every layer)."""
import pytest
import torch

from robustpointclouds_amd import _ffi

pytestmark = pytest.mark.gpu

# (gemm K = gathered row width, gemm N = output width): every launch shape of rpc_spconv_gemm_bf16
SHAPES = [(16, 16), (32, 16), (32, 32), (16, 32), (32, 64), (64, 32), (64, 64), (64, 128), (128, 64),
          (128, 128), (32, 128), (64, 16), (128, 32), (24, 32), (40, 64)]


def _r8(c):
    return (c + 7) // 8 * 8


def _run(lib, mode, a, n_src, kg, nbr, K, rev, n_out, bt, ng, epi, ez, ebn, dev):
    prev = lib.rpc_spconv_gemm_bf16_mode(mode)
    try:
        out = torch.full((n_out, ng), float("nan"), device=dev)
        nblk = max(lib.rpc_spconv_gemm_blocks(n_out), 1)
        part = torch.full((nblk, 2 * ng), float("nan"), device=dev) if epi != 2 else None
        _ffi.check(lib.rpc_spconv_gemm_bf16_n(_ffi.ptr(a), n_src, kg, _ffi.ptr(nbr), K, rev, n_out, _ffi.ptr(bt), ng,
                                              _ffi.ptr(out), _ffi.ptr(ez), _ffi.ptr(ebn), _ffi.ptr(part), epi,
                                              _ffi.stream_of(out)), "rpc_spconv_gemm_bf16_n")
        torch.cuda.synchronize()
        return out, part
    finally:
        lib.rpc_spconv_gemm_bf16_mode(prev)


@pytest.mark.parametrize("kg,ng", SHAPES)
@pytest.mark.parametrize("n_out,K,rev", [(5000, 27, 0), (129, 27, 1), (17, 3, 0), (15, 27, 0), (1, 27, 1)])
def test_pipe_gemm_bit_identical(kg, ng, n_out, K, rev):
    lib = _ffi.load()
    dev = torch.device("cuda")
    g = torch.Generator().manual_seed(kg * 131 + ng * 7 + n_out + K)
    n_src = 3000
    nbr = torch.randint(0, n_src, (n_out, K), generator=g, dtype=torch.int32)
    nbr[torch.rand((n_out, K), generator=g) > 0.35] = -1
    if K > 2:
        nbr[:, 1] = -1                      # an offset nobody uses
    if n_out > 300:
        nbr[128:256] = -1                   # a whole block of rows with no neighbour
    a = torch.zeros((n_src, _r8(kg)), dtype=torch.bfloat16)
    a[:, :kg] = torch.randn((n_src, kg), generator=g).to(torch.bfloat16)
    W = torch.randn((K, kg, ng), generator=g) * 0.1
    a, nbr, W = a.to(dev), nbr.to(dev), W.to(dev)
    bt = torch.empty(lib.rpc_spconv_bf16_weight_elems(K, kg, ng, 0), dtype=torch.bfloat16, device=dev)
    _ffi.check(lib.rpc_spconv_prep_weight_bf16(_ffi.ptr(W), K, kg, ng, 0, _ffi.ptr(bt), _ffi.stream_of(bt)), "prep")
    ez = torch.randn((n_out, ng), generator=g).to(dev)
    ebn = torch.cat([torch.rand(ng, generator=g) + 0.5, torch.randn(ng, generator=g) * 0.1,
                     torch.randn(ng, generator=g) * 0.1, torch.rand(ng, generator=g) + 0.5]).to(dev)
    for epi in (0, 1, 2):
        ref_out, ref_part = _run(lib, 0, a, n_src, kg, nbr, K, rev, n_out, bt, ng, epi, ez, ebn, dev)
        assert torch.isfinite(ref_out).all()
        for mode in (1, 2, 3):
            out, part = _run(lib, mode, a, n_src, kg, nbr, K, rev, n_out, bt, ng, epi, ez, ebn, dev)
            assert torch.equal(out, ref_out), (mode, epi)
            if epi != 2 and (kg, ng) == (128, 128):
                # k_gemm_bf16 runs the 128 x 128 tiles as two 16-row tiles per wave, the ring one (LDS):
                # the same rows per partial row, summed over 2 vs 4 waves
                assert torch.allclose(part, ref_part, rtol=1e-5, atol=1e-5), (mode, epi)
            elif epi != 2:
                assert torch.equal(part, ref_part), (mode, epi)


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


def _encoder_step(enc, feats, coors, mode, fused, perm=False, fmt=0):
    from robustpointclouds_amd import sparse_encoder as se
    lib = _ffi.load()
    prev, prev_f, prev_fmt, prev_p = lib.rpc_spconv_gemm_bf16_mode(mode), se.FUSED_FINALIZE, se.FWD_FMT, se.MASK_PERM
    prev_ff = se.FUSED_FINALIZE_FWD
    se.FUSED_FINALIZE = se.FUSED_FINALIZE_FWD = fused
    se.FWD_FMT = fmt   # 0: bf16 forward operands (the ring kernel is a bf16 path), 1: fp16 (the perf default)
    se.MASK_PERM = perm
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
        lib.rpc_spconv_gemm_bf16_mode(prev)
        se.FUSED_FINALIZE = prev_f
        se.FUSED_FINALIZE_FWD = prev_ff
        se.FWD_FMT = prev_fmt
        se.MASK_PERM = prev_p


def test_pipe_encoder_step_bit_identical():
    """The bf16 SparseEncoder forward + backward on a synthetic KITTI batch (the metric's shapes) with the
    ring kernel equals the one with the former kernel, bit for bit (dense BEV, every gradient, running stats),
    both with the separate BatchNorm finalize launches."""
    enc, feats, coors = _encoder_case()
    r0 = _encoder_step(enc, feats, coors, 0, False)
    r1 = _encoder_step(enc, feats, coors, 1, False)
    assert torch.equal(r0[0], r1[0])
    assert torch.equal(r0[1], r1[1])
    for a, b in zip(r0[2] + r0[3], r1[2] + r1[3]):
        assert torch.equal(a, b)


@pytest.mark.parametrize("mode,fmt", [(1, 0), (0, 0), (0, 1)])
def test_fused_finalize_matches_separate_and_is_deterministic(mode, fmt):
    """BatchNorm finalizes fused into the GEMMs (two-level last-block sums; forward on bf16 or fp16 operands,
    the ring or the regular kernel) against the separate rpc_bn_finalize launches: bit-identical from run to run,
    the ticket counters back at zero after every launch, and the same results up to the double-sum order of the
    statistics, whose last-bit differences could flip a bf16 rounding or a ReLU mask downstream (relative L2 <= 5e-2
    on the BEV, every gradient and the running statistics, the bound of the row-order test below; measured 0:
    bit-identical on this case, r04)."""
    enc, feats, coors = _encoder_case()
    ref = _encoder_step(enc, feats, coors, mode, False, fmt=fmt)
    a = _encoder_step(enc, feats, coors, mode, True, fmt=fmt)
    b = _encoder_step(enc, feats, coors, mode, True, fmt=fmt)
    for x, y in zip([a[0], a[1]] + a[2] + a[3], [b[0], b[1]] + b[2] + b[3]):
        assert torch.equal(x, y)
    worst = 0.0
    for i, (x, y) in enumerate(zip([ref[0], ref[1]] + ref[2] + ref[3], [a[0], a[1]] + a[2] + a[3])):
        d = ((x.double() - y.double()).norm() / max(y.double().norm().item(), 1e-30)).item()
        worst = max(worst, d)
        assert d < 5e-2, (i, d)
    print(f"fused vs separate finalize (mode {mode}, fmt {fmt}): worst relative L2 {worst:.2e}")
    assert int(enc.fin_tickets(feats.device).abs().sum().item()) == 0


@pytest.mark.parametrize("kg,ng,n_out,epi", [(64, 64, 106000, 0), (32, 64, 5000, 1), (64, 128, 130, 0),
                                             (128, 128, 64, 1), (16, 32, 1, 0)])
def test_gemm_fin_entry_point(kg, ng, n_out, epi):
    """rpc_spconv_gemm_bf16_fin alone: the same output rows as the unfused GEMM, the finalize outputs of
    rpc_bn_finalize on the same partial rows (mode 0: bn + running stats; mode 1: bnb, dgamma, dbeta) to
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
    nb = 4 if epi == 0 else 5
    for rep in range(3):
        out = torch.full((n_out, ng), float("nan"), device=dev)
        part = torch.full((nblk, 2 * ng), float("nan"), device=dev)
        rm0, rv0 = torch.zeros(ng, device=dev), torch.ones(ng, device=dev)
        rm, rv = rm0.clone(), rv0.clone()
        bn = torch.full((nb * ng,), float("nan"), device=dev)
        dg, db = torch.full((ng,), float("nan"), device=dev), torch.full((ng,), float("nan"), device=dev)
        fin = _ffi.RpcBnFin(ticket.data_ptr(), gpart.data_ptr(), epi, gamma.data_ptr(), beta.data_ptr(), 1e-3, 0.01,
                            rm.data_ptr(), rv.data_ptr(), ebn.data_ptr() if epi else None, bn.data_ptr(),
                            dg.data_ptr() if epi else None, db.data_ptr() if epi else None)
        _ffi.check(lib.rpc_spconv_gemm_bf16_fin(_ffi.ptr(a), n_src, kg, _ffi.ptr(nbr), K, 0, n_out, _ffi.ptr(bt), ng,
                                                _ffi.ptr(out), _ffi.ptr(ez) if epi else None,
                                                _ffi.ptr(ebn) if epi else None, _ffi.ptr(part), epi,
                                                _ffi.C.byref(fin), st), "rpc_spconv_gemm_bf16_fin")
        ref_out, ref_part = _run(lib, 0, a, n_src, kg, nbr, K, 0, n_out, bt, ng, epi, ez, ebn, dev)
        assert torch.equal(out, ref_out)
        assert torch.equal(part, ref_part)
        rrm, rrv = rm0.clone(), rv0.clone()
        rbn = torch.full((nb * ng,), float("nan"), device=dev)
        rdg, rdb = torch.full((ng,), float("nan"), device=dev), torch.full((ng,), float("nan"), device=dev)
        _ffi.check(lib.rpc_bn_finalize(_ffi.ptr(part), nblk, ng, n_out, epi, _ffi.ptr(gamma), _ffi.ptr(beta), 1e-3,
                                       0.01, _ffi.ptr(rrm), _ffi.ptr(rrv), _ffi.ptr(ebn) if epi else None,
                                       _ffi.ptr(rbn), _ffi.ptr(rdg) if epi else None, _ffi.ptr(rdb) if epi else None,
                                       None, st), "rpc_bn_finalize")
        torch.cuda.synchronize()
        pairs = [(bn, rbn)] + ([(rm, rrm), (rv, rrv)] if epi == 0 else [(dg, rdg), (db, rdb)])
        for x, y in pairs:
            assert torch.isfinite(x).all()
            assert torch.allclose(x, y, rtol=1e-6, atol=1e-6 * max(y.abs().max().item(), 1.0))
        assert int(ticket.abs().sum().item()) == 0


@pytest.mark.parametrize("n,K", [(5000, 27), (2048, 27), (1, 27), (70001, 3), (4099, 27)])
def test_mask_perm_orders_rows_by_mask(n, K):
    """rpc_rulebook_mask_perm: a permutation of the rows that, within every window of 2048 rows, lists them by
    neighbour mask (bit k = a neighbour at offset k), ties in row order — numpy's stable sort of the same keys."""
    import numpy as np
    lib = _ffi.load()
    dev = torch.device("cuda")
    g = torch.Generator().manual_seed(n + K)
    nbr = torch.randint(0, 100, (n, K), generator=g, dtype=torch.int32)
    nbr[torch.rand((n, K), generator=g) > 0.3] = -1
    nd = nbr.to(dev)
    perm = torch.full((n,), -7, dtype=torch.int32, device=dev)
    _ffi.check(lib.rpc_rulebook_mask_perm(_ffi.ptr(nd), n, K, _ffi.ptr(perm), _ffi.stream_of(perm)), "mask_perm")
    torch.cuda.synchronize()
    got = perm.cpu().numpy()
    mask = ((nbr.numpy() >= 0).astype(np.int64) << np.arange(K)).sum(1)
    want = np.concatenate([s + np.argsort(mask[s:s + 2048], kind="stable") for s in range(0, n, 2048)])
    assert np.array_equal(got, want)


@pytest.mark.parametrize("kg,ng", [(32, 32), (64, 64), (32, 64), (64, 32), (128, 128)])
def test_gemm_perm_writes_rows_in_place(kg, ng):
    """rpc_spconv_gemm_perm with the mask order: every output row equal to the natural order's (each row's own
    sums are unchanged; -0 == +0), forward / data gradient / plain; the BatchNorm partial rows sum to the same
    column totals (another grouping of the same values)."""
    lib = _ffi.load()
    dev = torch.device("cuda")
    g = torch.Generator().manual_seed(kg * 5 + ng)
    n_out, n_src, K = 9000, 6000, 27
    nbr = torch.randint(0, n_src, (n_out, K), generator=g, dtype=torch.int32)
    nbr[torch.rand((n_out, K), generator=g) > 0.3] = -1
    a = torch.zeros((n_src, _r8(kg)), dtype=torch.bfloat16)
    a[:, :kg] = torch.randn((n_src, kg), generator=g).to(torch.bfloat16)
    W = torch.randn((K, kg, ng), generator=g) * 0.1
    a, nbr, W = a.to(dev), nbr.to(dev), W.to(dev)
    bt = torch.empty(lib.rpc_spconv_bf16_weight_elems(K, kg, ng, 0), dtype=torch.bfloat16, device=dev)
    st = _ffi.stream_of(W)
    _ffi.check(lib.rpc_spconv_prep_weight_bf16(_ffi.ptr(W), K, kg, ng, 0, _ffi.ptr(bt), st), "prep")
    perm = torch.empty(n_out, dtype=torch.int32, device=dev)
    _ffi.check(lib.rpc_rulebook_mask_perm(_ffi.ptr(nbr), n_out, K, _ffi.ptr(perm), st), "mask_perm")
    ez = torch.randn((n_out, ng), generator=g).to(dev)
    ebn = torch.cat([torch.rand(ng, generator=g) + 0.5, torch.randn(ng, generator=g) * 0.1,
                     torch.randn(ng, generator=g) * 0.1, torch.rand(ng, generator=g) + 0.5]).to(dev)
    nblk = lib.rpc_spconv_gemm_blocks(n_out)
    for epi in (0, 1, 2):
        res = []
        for pm in (None, perm):
            out = torch.full((n_out, ng), float("nan"), device=dev)
            part = torch.full((nblk, 2 * ng), float("nan"), device=dev) if epi != 2 else None
            _ffi.check(lib.rpc_spconv_gemm_perm(_ffi.ptr(a), 0, n_src, kg, _ffi.ptr(nbr), K, 0, _ffi.ptr(pm), n_out,
                                                _ffi.ptr(bt), ng, _ffi.ptr(out), _ffi.ptr(ez), _ffi.ptr(ebn),
                                                _ffi.ptr(part), epi, st), "gemm_perm")
            torch.cuda.synchronize()
            res.append((out, part))
        assert torch.equal(res[0][0], res[1][0]), epi
        if epi != 2:
            t0, t1 = res[0][1].double().sum(0), res[1][1].double().sum(0)
            assert torch.allclose(t0, t1, rtol=1e-5, atol=1e-4 * float(t0.abs().max())), epi


def test_mask_order_encoder_step_close_and_deterministic():
    """The bf16 encoder step with the rows of every 16-bit GEMM in mask order against index order, and
    bit-identical from run to run. Every row's GEMM sum is unchanged (absent neighbours add exact zeros);
    the BatchNorm partial sums are grouped differently, so mean / var move in the last fp32 bits and some
    bf16-stored activations and gradients round one ulp the other way. With the bf16 forward operands this
    test runs (FWD_FMT = 0), each ordering is ~0.22 (relative L2) from float64 on the input gradient
    (tests/test_gpu_sparse_layers.py, perf_bf16fwd) and the two differ by 2.5e-2 there, 1.5e-3 on the
    BEV: bounded at 5e-2 — the mask order is as accurate as the index order (measured with the default
    fp16 forward: input gradient 7.37e-2 from float64 against the operand-emulation oracle's 7.39e-2)."""
    enc, feats, coors = _encoder_case()
    ref = _encoder_step(enc, feats, coors, 0, False, perm=False)
    a = _encoder_step(enc, feats, coors, 0, False, perm=True)
    b = _encoder_step(enc, feats, coors, 0, False, perm=True)
    for x, y in zip([a[0], a[1]] + a[2] + a[3], [b[0], b[1]] + b[2] + b[3]):
        assert torch.equal(x, y)
    worst = 0.0
    for i, (x, y) in enumerate(zip([ref[0], ref[1]] + ref[2] + ref[3], [a[0], a[1]] + a[2] + a[3])):
        d = ((x.double() - y.double()).norm() / max(y.double().norm().item(), 1e-30)).item()
        worst = max(worst, d)
        assert d < 5e-2, (i, d)
    print(f"mask order vs index order: worst relative L2 {worst:.2e}")


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
    din, _ = _run(lib, 0, a, n_src, kg, nbr, K, 0, n_out, bt, ng, 2, None, None, dev)
    m_ref = torch.full((n_out, ng), float("nan"), device=dev)
    p_ref = torch.full((nblk, 2 * ng), float("nan"), device=dev)
    _ffi.check(lib.rpc_sparse_res_backward(_ffi.ptr(gid) if g2 else _ffi.ptr(din), _ffi.ptr(din) if g2 else None,
                                           _ffi.ptr(out), _ffi.ptr(z), _ffi.ptr(bn), n_out, ng, _ffi.ptr(m_ref),
                                           _ffi.ptr(p_ref), st), "rpc_sparse_res_backward")
    # fused
    m = torch.full((n_out, ng), float("nan"), device=dev)
    p = torch.full((nblk, 2 * ng), float("nan"), device=dev)
    _ffi.check(lib.rpc_spconv_gemm_res(_ffi.ptr(a), n_src, kg, _ffi.ptr(nbr), K, 0, None, n_out, _ffi.ptr(bt), ng,
                                       _ffi.ptr(m), _ffi.ptr(gid) if g2 else None, _ffi.ptr(out), _ffi.ptr(z),
                                       _ffi.ptr(bn), _ffi.ptr(p), None, st), "rpc_spconv_gemm_res")
    torch.cuda.synchronize()
    assert torch.equal(m, m_ref)
    scale = torch.cat([m.abs().sum(0), (m * ((z - bn[2 * ng:3 * ng]) * bn[3 * ng:])).abs().sum(0)])
    assert torch.all((p.sum(0) - p_ref.sum(0)).abs() <= 1e-5 * scale + 1e-6)
