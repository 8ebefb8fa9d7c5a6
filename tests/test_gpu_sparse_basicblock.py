"""§8(f3): the basicblock SparseEncoder of the CenterPoint nuScenes base (SparseBasicBlock residual
stages, a stride-2 SparseConv3d closing each stage) on the HIP kernels vs the CPU float64 oracle,
forward and backward, on voxelised synthetic nuScenes sweeps (F = 5).

fp32 parity mode on a reduced-width stack (every fp32 width pair compiled); the full nuScenes widths
(up to 128 x 128) in the bf16 perf mode at bf16-level agreement."""
import numpy as np
import pytest
import torch

from oracle import voxelize as ov
from oracle.sparse_encoder import OracleSparseEncoder
from robustpointclouds_amd.sparse_encoder import SparseEncoder
from robustpointclouds_amd.synthetic import NUS_PC_RANGE, NUS_VOXEL_SIZE, nus_frame

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")
NUS_SHAPE = [41, 1024, 1024]


def _inputs(B, stride, seed=0, sweeps=2):
    frames = [nus_frame(seed + i, sweeps=sweeps)[::stride] for i in range(B)]
    vox, coors, npts = ov.voxelize_frames(frames, NUS_VOXEL_SIZE, NUS_PC_RANGE, 10, 90000)
    feats = vox[:, :, :5].sum(1) / npts[:, None]
    return feats.astype(np.float32), coors.astype(np.int32)


def _randomise_bn(enc):
    with torch.no_grad():
        for m in enc.layers():
            m[1].weight.uniform_(0.5, 1.5)
            m[1].bias.uniform_(-0.2, 0.2)


def test_structure_and_names():
    enc = SparseEncoder(5, NUS_SHAPE, output_channels=128,
                        encoder_channels=((16, 16, 32), (32, 32, 64), (64, 64, 128), (128, 128)),
                        encoder_paddings=((0, 0, 1), (0, 0, 1), (0, 0, [0, 1, 1]), (1, 1)), block_type="basicblock")
    assert enc.shapes == [(41, 1024, 1024), (21, 512, 512), (11, 256, 256), (5, 128, 128), (2, 128, 128)]
    assert len(enc.specs) == 21 and enc.specs[-1].co == 128
    keys = set(enc.state_dict().keys())
    for k in ("encoder_layers.encoder_layer1.0.conv1.weight", "encoder_layers.encoder_layer1.0.bn2.running_var",
              "encoder_layers.encoder_layer1.2.0.weight", "encoder_layers.encoder_layer4.1.conv2.weight",
              "conv_out.1.weight"):
        assert k in keys, k
    mats = [i for i, s in enumerate(enc.specs) if s.mat]
    assert mats == [0, 2, 4, 5, 7, 9, 10, 12, 14, 15, 17, 19]
    assert [s.res for s in enc.specs if s.res >= 0] == [0, 2, 5, 7, 10, 12, 15, 17]


def test_basicblock_fp32_matches_oracle():
    torch.manual_seed(0)
    B = 2
    feats, coors = _inputs(B, stride=6)
    enc = SparseEncoder(5, NUS_SHAPE, output_channels=64, encoder_channels=((16, 16, 32), (32, 32, 64), (64, 64)),
                        encoder_paddings=((0, 0, 1), (0, 0, 1), (1, 1)), block_type="basicblock").to(DEV)
    _randomise_bn(enc)
    orc = OracleSparseEncoder(enc)
    f = torch.from_numpy(feats).to(DEV).requires_grad_(True)
    out = enc(f, torch.from_numpy(coors).to(DEV), B)
    ref_f = torch.from_numpy(feats).double().requires_grad_(True)
    ref = orc.forward(ref_f, coors, B)
    assert out.shape == ref.shape
    o = out.detach().cpu().double()
    err, scale = (o - ref.detach()).abs().max().item(), ref.abs().max().item()
    assert err <= 1e-4 * max(scale, 1.0), (err, scale)
    for m, p in zip(enc.layers(), orc.params):
        np.testing.assert_allclose(m[1].running_mean.cpu().numpy(), p["rm"].numpy(), rtol=1e-4, atol=1e-5)
    G = torch.randn(out.shape, generator=torch.Generator().manual_seed(1))
    (out * G.to(DEV)).sum().backward()
    (ref * G.double()).sum().backward()

    # 16 train-mode BatchNorm backwards in fp32 with residual sums on top (the SECOND stack has 12 and
    # meets 1e-3 / 2e-3): relative L2 <= 2e-3 and every element within 5e-3 of the max
    def close(got, want, name):
        got = got.cpu().double()
        rel = ((got - want).norm() / want.norm().clamp_min(1e-30)).item()
        mx = (got - want).abs().max().item() / max(want.abs().max().item(), 1e-30)
        assert rel <= 2e-3 and mx <= 5e-3, (name, rel, mx)

    close(f.grad, ref_f.grad, "feats")
    for i, (m, p) in enumerate(zip(enc.layers(), orc.params)):
        close(m[0].weight.grad, p["W"].grad, f"W{i}")
        close(m[1].weight.grad, p["g"].grad, f"gamma{i}")
        close(m[1].bias.grad, p["b"].grad, f"beta{i}")


def test_basicblock_nuscenes_bf16_close_to_oracle():
    torch.manual_seed(0)
    B = 1
    feats, coors = _inputs(B, stride=4)
    enc = SparseEncoder(5, NUS_SHAPE, output_channels=128,
                        encoder_channels=((16, 16, 32), (32, 32, 64), (64, 64, 128), (128, 128)),
                        encoder_paddings=((0, 0, 1), (0, 0, 1), (0, 0, [0, 1, 1]), (1, 1)),
                        block_type="basicblock").to(DEV)
    enc.bf16 = True
    orc = OracleSparseEncoder(enc)
    f = torch.from_numpy(feats).to(DEV).requires_grad_(True)
    out = enc(f, torch.from_numpy(coors).to(DEV), B)
    ref_f = torch.from_numpy(feats).double().requires_grad_(True)
    ref = orc.forward(ref_f, coors, B)
    assert out.shape == ref.shape == (B, 256, 128, 128)
    rel = ((out.detach().cpu().double() - ref.detach()).norm() / ref.norm()).item()
    assert rel < 3e-2, rel
    G = torch.randn(out.shape, generator=torch.Generator().manual_seed(1))
    (out * G.to(DEV)).sum().backward()
    (ref * G.double()).sum().backward()
    cos = lambda a, b: (a.flatten() @ b.flatten() / (a.norm() * b.norm())).item()
    assert cos(f.grad.cpu().double(), ref_f.grad) > 0.95
    for i, (m, p) in enumerate(zip(enc.layers(), orc.params)):
        c = cos(m[0].weight.grad.cpu().double(), p["W"].grad)
        assert c > 0.95, (i, c)


def test_fused_residual_backward_matches_separate():
    """The bf16 basicblock encoder's backward with the residual backward fused into the data-gradient GEMMs
    (rpc_sparse_tune knob 0 = 1, the default) against the separate rpc_sparse_res_backward passes: the m rows
    are the same, the BatchNorm-backward partial sums are added in another order, and a last-bit difference there
    moves bf16 roundings and ReLU decisions downstream — every gradient within relative L2 5e-2 of the separate
    path (the bound of the row-order test, tests/test_gpu_sparse_pipe.py; measured 6.4e-3 on the input gradient),
    the input gradient as close to the float64 oracle as the separate path's, bit-identical from run to run."""
    from robustpointclouds_amd import _ffi
    lib = _ffi.load()
    torch.manual_seed(0)
    B = 1
    feats, coors = _inputs(B, stride=4)
    enc = SparseEncoder(5, NUS_SHAPE, output_channels=128,
                        encoder_channels=((16, 16, 32), (32, 32, 64), (64, 64, 128), (128, 128)),
                        encoder_paddings=((0, 0, 1), (0, 0, 1), (0, 0, [0, 1, 1]), (1, 1)),
                        block_type="basicblock").to(DEV)
    enc.bf16 = True
    G = torch.randn((B, 256, 128, 128), generator=torch.Generator().manual_seed(1)).to(DEV)
    bns = [m[1] for m in enc.layers()]
    saved = [(b.running_mean.clone(), b.running_var.clone()) for b in bns]

    def step(fuse):
        old = lib.rpc_sparse_tune(0, fuse)
        try:
            for q in enc.parameters():
                q.grad = None
            for b, (mm, vv) in zip(bns, saved):
                b.running_mean.copy_(mm)
                b.running_var.copy_(vv)
            f = torch.from_numpy(feats).to(DEV).requires_grad_(True)
            out = enc(f, torch.from_numpy(coors).to(DEV), B)
            (out * G).sum().backward()
            torch.cuda.synchronize()
            return [f.grad.clone()] + [q.grad.clone() for q in enc.parameters()]
        finally:
            lib.rpc_sparse_tune(0, old)

    sep, fa, fb = step(0), step(1), step(1)
    for x, y in zip(fa, fb):
        assert torch.equal(x, y)
    worst = 0.0
    for i, (x, y) in enumerate(zip(fa, sep)):
        d = ((x.double() - y.double()).norm() / y.double().norm().clamp_min(1e-30)).item()
        worst = max(worst, d)
        assert d <= 5e-2, (i, d)
    print(f"fused vs separate residual backward: worst relative L2 {worst:.2e}")
    orc = OracleSparseEncoder(enc)
    ref_f = torch.from_numpy(feats).double().requires_grad_(True)
    (orc.forward(ref_f, coors, B) * G.cpu().double()).sum().backward()
    rel = lambda x: ((x.cpu().double() - ref_f.grad).norm() / ref_f.grad.norm()).item()
    ef, es = rel(fa[0]), rel(sep[0])
    print(f"input gradient vs float64: fused {ef:.3e}, separate {es:.3e}")
    assert ef <= 1.1 * es + 1e-3, (ef, es)
