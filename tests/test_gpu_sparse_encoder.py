"""a6 parity: HIP SparseEncoder (rulebooks + implicit-GEMM convs + BN + dense) against the
CPU float64 oracle, forward and backward, on voxelised synthetic KITTI frames."""
import numpy as np
import pytest
import torch

from oracle import voxelize as ov
from oracle.sparse_encoder import OracleSparseEncoder, implementation_masks, spconv_pairs, subm_pairs
from robustpointclouds_amd.sparse_encoder import SparseEncoder
from robustpointclouds_amd.synthetic import KITTI_PC_RANGE, KITTI_VOXEL_SIZE, kitti_frame
from tests._dense_masks import FlipStats

pytestmark = pytest.mark.gpu
FLIP_PRE_MAX = 1e-4   # an adopted ReLU decision float64 takes differently lies within this of 0 (x channel max |act|)


def _inputs(B, stride=3, seed=0):
    frames = [kitti_frame(seed + i)[::stride] for i in range(B)]
    vox, coors, npts = ov.voxelize_frames(frames, KITTI_VOXEL_SIZE, KITTI_PC_RANGE, 5, 16000)
    feats = vox[:, :, :4].sum(1) / npts[:, None]
    return feats.astype(np.float32), coors.astype(np.int32)


BASIC = dict(output_channels=128, encoder_channels=((16, 16, 32), (32, 32, 64), (64, 64, 128), (128, 128)),
             encoder_paddings=((0, 0, 1), (0, 0, 1), (0, 0, [0, 1, 1]), (1, 1)), block_type="basicblock")


@pytest.mark.parametrize("B,stride,basic", [(2, 4, False), (1, 1, False), (1, 4, True), (1, 4, "nus")])
def test_sparse_encoder_forward_backward_matches_oracle(B, stride, basic):
    """basic: the CenterPoint basicblock encoder (residual SparseBasicBlocks, 128-wide fp32 convs);
    "nus": the same with CenterPoint's 5 input features (conv_input 5 -> 16, its 5-wide data gradient)."""
    torch.manual_seed(0)
    feats, coors = _inputs(B, stride)
    if basic == "nus":
        feats = np.concatenate([feats, np.random.default_rng(4).uniform(0, 0.5, (len(feats), 1))], 1).astype(np.float32)
    dev = torch.device("cuda")
    enc = SparseEncoder(feats.shape[1], [41, 1600, 1408], **(BASIC if basic else {})).to(dev)
    with torch.no_grad():   # non-trivial BN affine params
        for m in enc.layers():
            m[1].weight.uniform_(0.5, 1.5)
            m[1].bias.uniform_(-0.2, 0.2)
    orc = OracleSparseEncoder(enc)
    f = torch.from_numpy(feats).to(dev).requires_grad_(True)
    enc.debug = []
    out = enc(f, torch.from_numpy(coors).to(dev), B)
    G = torch.randn(out.shape, generator=torch.Generator().manual_seed(1))
    (out * G.to(dev)).sum().backward()
    # the float64 oracle on the HIP encoder's ReLU decisions (oracle/sparse_encoder.py `masks`): an fp32
    # pre-activation within a rounding of 0 falls on either side, and one on the other side moved beta6 by
    # 3e-3 of its max (r05, after the fp32 GEMM's two-level sums changed the rounding)
    masks = implementation_masks(enc.debug)
    enc.debug = None
    ref_f = torch.from_numpy(feats).double().requires_grad_(True)
    flips = FlipStats()
    ref = orc.forward(ref_f, coors, B, masks=masks, flips=flips)
    print(f"sparse ReLU decisions differing from float64's: {flips.flips} (max |act| {flips.worst:.1e} of channel "
          f"max; per layer {flips.per_layer})")
    assert flips.worst <= FLIP_PRE_MAX, flips
    assert out.shape == ref.shape == (B, 256, 200, 176)
    o = out.detach().cpu().double()
    scale = ref.abs().max().item()
    assert (o - ref.detach()).abs().max().item() <= 1e-4 * max(scale, 1.0)
    # running stats
    for m, p in zip(enc.layers(), orc.params):
        np.testing.assert_allclose(m[1].running_mean.cpu().numpy(), p["rm"].numpy(), rtol=1e-4, atol=1e-5)
        np.testing.assert_allclose(m[1].running_var.cpu().numpy(), p["rv"].numpy(), rtol=1e-3, atol=1e-5)
    (ref * G.double()).sum().backward()
    # gradients pass through 12 train-mode BatchNorm backwards (mean-subtracting, so fp32
    # cancellation; fp32 sums over ~1e4 rows x 27 offsets): relative L2 error <= 1e-3 and
    # every element within 2e-3 of the max
    def close(got, want, name):
        got = got.cpu().double()
        rel = ((got - want).norm() / want.norm().clamp_min(1e-30)).item()
        mx = (got - want).abs().max().item() / max(want.abs().max().item(), 1e-30)
        assert rel <= 1e-3 and mx <= 2e-3, (name, rel, mx)
    close(f.grad, ref_f.grad, "feats")
    for i, (m, p) in enumerate(zip(enc.layers(), orc.params)):
        close(m[0].weight.grad, p["W"].grad, f"W{i}")
        close(m[1].weight.grad, p["g"].grad, f"gamma{i}")
        close(m[1].bias.grad, p["b"].grad, f"beta{i}")


def test_rulebooks_match_oracle_pairs():
    feats, coors = _inputs(2, 5)
    dev = torch.device("cuda")
    enc = SparseEncoder(4, [41, 1600, 1408]).to(dev)
    out = enc(torch.from_numpy(feats).to(dev), torch.from_numpy(coors).to(dev), 2)
    # deterministic: the same input gives the same bytes
    out2 = enc(torch.from_numpy(feats).to(dev), torch.from_numpy(coors).to(dev), 2)
    # (BN running stats moved, but the batch-stat forward output does not depend on them)
    assert torch.equal(out, out2)
    # grids are left clean (all -1) after use
    for g in enc._grids.values():
        assert int((g != -1).sum().item()) == 0
    # pair counts per offset of the first SubM and the first strided conv
    c = coors.astype(np.int64)
    sub = subm_pairs(c, (2, 41, 1600, 1408))
    assert sum(len(a) for a, _ in sub) > 0
    oc, sp = spconv_pairs(c, (2, 21, 800, 704), (3, 3, 3), (2, 2, 2), (1, 1, 1))
    assert oc.shape[0] > 0


def test_bf16_perf_mode_close_to_oracle():
    """bf16 MFMA forward/dgrad (fp32 accumulate + fp32 BN statistics): bf16-level agreement."""
    torch.manual_seed(0)
    feats, coors = _inputs(2, 3)
    dev = torch.device("cuda")
    enc = SparseEncoder(4, [41, 1600, 1408]).to(dev)
    enc.bf16 = True
    orc = OracleSparseEncoder(enc)
    f = torch.from_numpy(feats).to(dev).requires_grad_(True)
    out = enc(f, torch.from_numpy(coors).to(dev), 2)
    ref_f = torch.from_numpy(feats).double().requires_grad_(True)
    ref = orc.forward(ref_f, coors, 2)
    rel = ((out.detach().cpu().double() - ref.detach()).norm() / ref.norm()).item()
    assert rel < 3e-2, rel
    G = torch.randn(out.shape, generator=torch.Generator().manual_seed(1))
    (out * G.to(dev)).sum().backward()
    (ref * G.double()).sum().backward()
    cos = lambda a, b: (a.flatten() @ b.flatten() / (a.norm() * b.norm())).item()
    # gradients of the bf16 forward (ReLU masks flip near 0): direction, not bits
    assert cos(f.grad.cpu().double(), ref_f.grad) > 0.95
    for i, (m, p) in enumerate(zip(enc.layers(), orc.params)):
        c = cos(m[0].weight.grad.cpu().double(), p["W"].grad)
        assert c > 0.95, (i, c)


@pytest.mark.parametrize("nhwc,bf16", [(True, False), (False, True), (True, True)])
def test_dense_image_layouts(nhwc, bf16):
    """channels_last / bf16 dense hand-over == the NCHW fp32 image (bf16: rounded), and the
    gradient path reads the same image layout back."""
    feats, coors = _inputs(2, 4)
    dev = torch.device("cuda")
    enc = SparseEncoder(4, [41, 1600, 1408]).to(dev)
    f = torch.from_numpy(feats).to(dev)
    c = torch.from_numpy(coors).to(dev)
    f0 = f.clone().requires_grad_(True)
    ref = enc(f0, c, 2)
    enc.dense_nhwc, enc.dense_bf16 = nhwc, bf16
    f1 = f.clone().requires_grad_(True)
    out = enc(f1, c, 2)
    assert out.shape == ref.shape and out.dtype == (torch.bfloat16 if bf16 else torch.float32)
    assert out.is_contiguous(memory_format=torch.channels_last) == nhwc
    want = ref.detach().to(out.dtype).float()
    assert torch.equal(out.detach().float(), want)
    G = torch.randn(ref.shape, generator=torch.Generator().manual_seed(3)).to(dev)
    if bf16:
        G = G.to(torch.bfloat16).float()   # exactly representable either way
    (ref * G).sum().backward()
    (out.float() * G).sum().backward()
    rel = ((f1.grad - f0.grad).norm() / f0.grad.norm()).item()
    assert rel < (1e-5 if not bf16 else 3e-2), rel


def test_bf16_perf_mode_config_size():
    """The bench's sparse encoder at the config size: 6 full synthetic KITTI frames (no subsample,
    16000-voxel cap), bf16 MFMA layers 1-11 (fp32 layer 0, fp32 accumulation and BN statistics),
    against the float64 oracle. Bounds (bf16 operands; measured at B=2 / stride 3: forward 2.4e-2,
    cosines > 0.97): forward relative L2 <= 3e-2; input and every weight gradient cosine >= 0.95;
    and the fp32 mode of the same layers on the same input <= 1e-4 (forward, max-normalised)."""
    torch.manual_seed(0)
    feats, coors = _inputs(6, 1, seed=20)
    dev = torch.device("cuda")
    enc = SparseEncoder(4, [41, 1600, 1408]).to(dev)
    orc = OracleSparseEncoder(enc)
    ref_f = torch.from_numpy(feats).double().requires_grad_(True)
    ref = orc.forward(ref_f, coors, 6)
    G = torch.randn(ref.shape, generator=torch.Generator().manual_seed(2))
    (ref * G.double()).sum().backward()
    c = torch.from_numpy(coors).to(dev)
    # fp32 mode
    out32 = enc(torch.from_numpy(feats).to(dev), c, 6)
    scale = ref.abs().max().item()
    assert (out32.cpu().double() - ref.detach()).abs().max().item() <= 1e-4 * max(scale, 1.0)
    # bf16 perf mode
    enc.bf16 = True
    f = torch.from_numpy(feats).to(dev).requires_grad_(True)
    out = enc(f, c, 6)
    rel = ((out.detach().cpu().double() - ref.detach()).norm() / ref.norm()).item()
    (out * G.to(dev)).sum().backward()
    cos = lambda a, b: (a.flatten() @ b.flatten() / (a.norm() * b.norm())).item()
    cf = cos(f.grad.cpu().double(), ref_f.grad)
    cw = [cos(m[0].weight.grad.cpu().double(), p["W"].grad) for m, p in zip(enc.layers(), orc.params)]
    print(f"B=6 bf16 sparse encoder: forward rel {rel:.3e}, dfeat cos {cf:.4f}, worst dW cos {min(cw):.4f}")
    assert rel < 3e-2, rel
    assert cf >= 0.95 and min(cw) >= 0.95, (cf, cw)


@pytest.mark.parametrize("bf16,basic", [(True, False), (False, False), (True, True), (False, True)])
def test_native_backward_bit_identical_to_layer_loop(bf16, basic):
    """rpc_sparse_backward (one C++ loop, weight gradients on the side stream) issues the same kernels
    with the same arguments in the same order as the per-layer Python loop: identical bits for the
    input gradient and every parameter gradient, conv_module and basicblock encoders, both precisions."""
    import robustpointclouds_amd.sparse_encoder as se
    dev = torch.device("cuda")
    feats, coors = _inputs(2, 2, seed=3)
    if basic:
        kw = dict(output_channels=128, encoder_channels=((16, 16, 32), (32, 32, 64), (64, 64, 128), (128, 128)),
                  encoder_paddings=((0, 0, 1), (0, 0, 1), (0, 0, [0, 1, 1]), (1, 1)), block_type="basicblock")
    else:
        kw = {}
    torch.manual_seed(0)
    enc = SparseEncoder(4, [41, 1600, 1408], **kw).to(dev)
    enc.bf16 = enc.dense_bf16 = bf16
    enc.dense_nhwc = bf16
    G = torch.randn((2, enc.output_channels * 2, 200, 176), generator=torch.Generator().manual_seed(2)).to(dev)
    res = {}
    saved = se.NATIVE_BACKWARD
    try:
        for native in (False, True):
            se.NATIVE_BACKWARD = native
            for p in enc.parameters():
                p.grad = None
            f = torch.from_numpy(feats).to(dev).requires_grad_(True)
            out = enc(f, torch.from_numpy(coors).to(dev), 2)
            (out.float() * G).sum().backward()
            torch.cuda.synchronize()
            res[native] = [f.grad.clone()] + [p.grad.clone() for p in enc.parameters()]
    finally:
        se.NATIVE_BACKWARD = saved
    for i, (a, b) in enumerate(zip(res[False], res[True])):
        assert torch.equal(a, b), i


@pytest.mark.parametrize("bf16", [False, True])
def test_dense_buffer_cleared_between_steps(bf16):
    """The persistent dense BEV buffer is cleared where the previous step scattered (rpc_sparse_dense_clear),
    not zero-filled whole: a step after a step on other voxels equals the same step on a fresh buffer,
    bit for bit."""
    torch.manual_seed(0)
    dev = torch.device("cuda")
    enc = SparseEncoder(4, [41, 1600, 1408]).to(dev)
    enc.bf16 = bf16
    fa, ca = _inputs(2, 3, seed=0)
    fb, cb = _inputs(2, 3, seed=7)
    enc(torch.from_numpy(fa).to(dev), torch.from_numpy(ca).to(dev), 2)
    got = enc(torch.from_numpy(fb).to(dev), torch.from_numpy(cb).to(dev), 2).clone()
    enc.__dict__.pop("_dense_bufs")
    want = enc(torch.from_numpy(fb).to(dev), torch.from_numpy(cb).to(dev), 2)
    assert torch.equal(got, want)   # (a cell of the first step left behind would differ from the fresh zeros)


@pytest.mark.parametrize("C,flags", [(6, 0), (6, 1), (6, 3), (8, 2)])
def test_dense_clear_any_width(C, flags):
    """rpc_sparse_dense_clear for output widths that are not a multiple of 4 (its scalar form) and the
    vector form: exactly the cells of the given coordinates (every channel, NCHW [B][C*D][H][W] or NHWC
    [B][H][W][C*D]) become 0, every other cell keeps its value."""
    from robustpointclouds_amd import _ffi
    dev = torch.device("cuda")
    B, D, H, W = 2, 2, 9, 7
    rng = np.random.default_rng(C + flags)
    cells = rng.choice(B * D * H * W, 23, replace=False)
    b, r = np.divmod(cells, D * H * W)
    z, r = np.divmod(r, H * W)
    y, x = np.divmod(r, W)
    coors = torch.from_numpy(np.stack([b, z, y, x], 1).astype(np.int32)).to(dev)
    dt = torch.bfloat16 if flags & 2 else torch.float32
    nhwc = bool(flags & 1)
    dense = torch.arange(1, B * C * D * H * W + 1, dtype=torch.float32).to(dt).to(dev)
    dense = dense.view((B, H, W, C * D) if nhwc else (B, C * D, H, W))
    want = dense.clone()
    for bi, zi, yi, xi in zip(b, z, y, x):
        for c in range(C):
            if nhwc:
                want[bi, yi, xi, c * D + zi] = 0
            else:
                want[bi, c * D + zi, yi, xi] = 0
    lib = _ffi.load()
    st = _ffi.stream_of(dense)
    _ffi.check(lib.rpc_sparse_dense_clear(_ffi.ptr(coors), len(cells), C, _ffi.int_arr((B, D, H, W)), flags,
                                          _ffi.ptr(dense), st), "clear")
    torch.cuda.synchronize()
    assert torch.equal(dense, want)
