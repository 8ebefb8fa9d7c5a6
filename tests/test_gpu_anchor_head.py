"""§8(f1) / row a8: Anchor3DHead targets + losses on the HIP kernels vs the CPU restatement.

Kernel level (rpc_anchor_head_loss_forward/backward through HeadLossFn): on the same head outputs
z (fp32 NCHW, or the bf16 NHWC GEMM image) and the same anchor tables, the per-anchor assignment
must equal oracle/anchor_head.py exactly (IoU / thresholds are bit-identical), the three losses and
num_total_pos must match the float64 oracle within 1e-4 relative (north_star fp32 tolerance), and
d loss / d z, d loss / d bias within 1e-4 relative-L2 (fp32 z) or bf16 rounding of dz (bf16 z).
Module level: Anchor3DHead.loss (HIP 1x1 GEMM in bf16 / torch conv in fp32 + HIP loss) against
float64 autograd of the oracle on the same bf16-rounded inputs.
Oracle parity w.r.t. upstream mmdet3d is unpinned (not vendored); see oracle/anchor_head.py.
"""
import numpy as np
import pytest
import torch

from oracle import anchor_head as oh
from robustpointclouds_amd.anchor_head import Anchor3DHead, HeadLossFn, pack_gt
from robustpointclouds_amd.synthetic import kitti_batch
from robustpointclouds_amd.voxelnet import second_kitti_cfg

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


def _head(num_classes, assign_per_class=False):
    cfg = second_kitti_cfg(num_classes)
    hc = dict(cfg["bbox_head"])
    hc.pop("type")
    hc.update(train_cfg=cfg["train_cfg"], test_cfg=cfg["test_cfg"], assign_per_class=assign_per_class)
    torch.manual_seed(0)
    return Anchor3DHead(**hc).to(DEV)


def _ocfg(head):
    return oh.cfg_of(head)


def _gt(B, num_classes, seed, H, W, empty=(), many=False):
    """Synthetic GT boxes; on a reduced map the boxes are placed inside its anchor range."""
    _, boxes, labels = kitti_batch(B, seed0=seed, num_classes=num_classes)
    samples = []
    rng = np.random.default_rng(seed)
    for b in range(B):
        bx, lb = np.asarray(boxes[b], np.float32), np.asarray(labels[b], np.int64)
        if many:
            k = 40
            idx = rng.integers(0, len(bx), k)
            bx = bx[idx] + rng.normal(0, 0.3, (k, 7)).astype(np.float32) * np.array([1, 1, 0, 0, 0, 0, 1], np.float32)
            lb = lb[idx]
        if b in empty:
            bx, lb = bx[:0], lb[:0]
        samples.append((bx, lb))
    return pack_gt(samples, DEV)


def _z(head, B, H, W, bf16, seed):
    g = torch.Generator().manual_seed(seed)
    A, C = head.num_anchors, head.num_classes
    N = A * (C + 9)
    z = torch.randn(B, N, H, W, generator=g) * 0.5
    z[:, :A * C] -= 4.0   # logits near the prior of the cls bias
    if bf16:
        zi = torch.zeros(B * H * W, 128, dtype=torch.bfloat16)
        zi[:, :N] = z.permute(0, 2, 3, 1).reshape(-1, N).to(torch.bfloat16)
        lay = dict(B=B, H=H, W=W, bf16=1, sb=H * W * 128, shw=128, sn=1, nwrite=128)
        zref = zi[:, :N].double().view(B, H, W, N).permute(0, 3, 1, 2).contiguous()
        return zi.to(DEV), lay, zref
    lay = dict(B=B, H=H, W=W, bf16=0, sb=N * H * W, shw=1, sn=H * W, nwrite=N)
    return z.contiguous().to(DEV), lay, z.double()


def _oracle(head, zref, bias, gb, gl, H, W):
    cfg = _ocfg(head)
    g = head.prior_generator
    anchors = oh.grid_anchors(H, W, g.ranges, g.sizes, g.rotations).double()
    zr = zref.clone().requires_grad_(True)
    br = bias.detach().cpu().double().clone().requires_grad_(True)
    out = oh.head_losses_from_z(cfg, zr, br, anchors, gb.cpu().double(), gl.cpu())
    return out, zr, br


CASES = [
    # (classes, assign_per_class, H, W, B, bf16, empty frames, many gts)
    (1, False, 200, 176, 2, False, (), False),
    (1, False, 200, 176, 2, True, (), False),
    (3, False, 200, 176, 2, False, (), False),
    (3, False, 200, 176, 2, True, (), False),
    (3, True, 200, 176, 2, False, (), False),
    (1, False, 200, 176, 3, False, (1,), False),
    (3, False, 200, 176, 2, False, (0, 1), False),
    (3, False, 200, 176, 2, False, (), True),
]


@pytest.mark.parametrize("case", CASES, ids=[f"c{c[0]}_apc{int(c[1])}_{'bf16' if c[5] else 'fp32'}_e{len(c[6])}"
                                               f"{'_many' if c[7] else ''}" for c in CASES])
def test_head_loss_kernel_vs_oracle(case):
    C, apc, H, W, B, bf16, empty, many = case
    head = _head(C, apc)
    gb, gl = _gt(B, C, 11 + B, H, W, empty, many)
    z, lay, zref = _z(head, B, H, W, bf16, seed=5)
    _, bias = head._stacked()
    bias = (bias.detach() + 0.1 * torch.randn_like(bias)).requires_grad_(True)
    zg = z.clone().requires_grad_(True)
    l3, asg, npos = HeadLossFn.apply(zg, bias, head, lay, gb, gl)
    ref, zr, br = _oracle(head, zref, bias, gb, gl, H, W)
    # assignment: exact
    np.testing.assert_array_equal(asg.cpu().numpy(), ref["assigned"].numpy().astype(np.int32))
    assert float(npos) == float(ref["num_total_pos"])
    got = l3.detach().cpu().double().numpy()
    want = np.array([float(ref["loss_cls"]), float(ref["loss_bbox"]), float(ref["loss_dir"])])
    np.testing.assert_allclose(got, want, rtol=1e-4, atol=1e-7)
    # gradients: weights != 1 on the three losses exercise the per-loss scaling
    w = torch.tensor([1.0, 0.7, 1.3])
    (l3 * w.to(DEV)).sum().backward()
    (ref["loss_cls"] * 1.0 + ref["loss_bbox"] * 0.7 + ref["loss_dir"] * 1.3).backward()
    N = zref.shape[1]
    if bf16:
        dz = zg.grad.float().cpu()[:, :N].double().view(B, H, W, N).permute(0, 3, 1, 2)
        assert torch.count_nonzero(zg.grad[:, N:]) == 0
        tol = 8e-3   # dz stored as bf16
    else:
        dz = zg.grad.double().cpu()
        tol = 1e-4
    rel = (dz - zr.grad).norm() / zr.grad.norm().clamp(min=1e-30)
    assert rel < tol, float(rel)
    assert (dz - zr.grad).abs().max() <= tol * zr.grad.abs().max() + 1e-12
    relb = (bias.grad.double().cpu() - br.grad).norm() / br.grad.norm()
    assert relb < max(tol, 1e-4), float(relb)


def test_head_loss_deterministic():
    head = _head(3)
    gb, gl = _gt(2, 3, 3, 200, 176)
    z, lay, _ = _z(head, 2, 200, 176, True, seed=1)
    _, bias = head._stacked()
    outs = []
    for _ in range(2):
        zg = z.clone().requires_grad_(True)
        b = bias.detach().clone().requires_grad_(True)
        l3, _, _ = HeadLossFn.apply(zg, b, head, lay, gb, gl)
        l3.sum().backward()
        outs.append((l3.detach().cpu(), zg.grad.cpu(), b.grad.cpu()))
    for a, b in zip(outs[0], outs[1]):
        assert torch.equal(a, b)


@pytest.mark.parametrize("classes", [1, 3])
@pytest.mark.parametrize("bf16", [False, True])
def test_anchor3dhead_module_vs_oracle(classes, bf16):
    """Anchor3DHead.loss end to end (1x1 GEMM + HIP loss), grads w.r.t. x, W, b."""
    head = _head(classes)
    B, Cin, H, W = 2, 512, 200, 176
    gb, gl = _gt(B, classes, 21, H, W)
    g = torch.Generator().manual_seed(3)
    x = torch.relu(torch.randn(B, Cin, H, W, generator=g))
    if bf16:
        x = x.to(torch.bfloat16)
        with torch.no_grad():
            for c in head._convs():
                c.weight.copy_(c.weight.to(torch.bfloat16).float())
    xd = x.to(DEV)
    if bf16:
        xd = xd.contiguous(memory_format=torch.channels_last)
    xd.requires_grad_(True)
    losses = head.loss([xd], dict(gt_boxes=gb, gt_labels=gl))
    total = sum(v[0] for v in losses.values())
    total.backward()
    # float64 reference on the same (bf16-rounded) values
    cfg = _ocfg(head)
    gen = head.prior_generator
    anchors = oh.grid_anchors(H, W, gen.ranges, gen.sizes, gen.rotations).double()
    xr = x.double().requires_grad_(True)
    convs = head._convs()
    wr = torch.cat([c.weight.detach().cpu().double() for c in convs]).requires_grad_(True)
    br = torch.cat([c.bias.detach().cpu().double() for c in convs]).requires_grad_(True)
    zr = torch.nn.functional.conv2d(xr, wr)
    ref = oh.head_losses_from_z(cfg, zr, br, anchors, gb.cpu().double(), gl.cpu())
    (ref["loss_cls"] + ref["loss_bbox"] + ref["loss_dir"]).backward()
    # bf16: z is rounded to bf16 before the loss (as under torch autocast): 1e-2 on values
    rtol = 1e-2 if bf16 else 1e-4
    for k in ("loss_cls", "loss_bbox", "loss_dir"):
        np.testing.assert_allclose(float(losses[k][0]), float(ref[k]), rtol=rtol, atol=1e-6)
    gw = torch.cat([c.weight.grad.detach().cpu().double() for c in convs])
    gbias = torch.cat([c.bias.grad.detach().cpu().double() for c in convs])
    gx = xd.grad.detach().float().cpu().double()
    for got, want, name in ((gx, xr.grad, "dx"), (gw, wr.grad, "dW"), (gbias, br.grad, "db")):
        rel = float((got - want).norm() / want.norm().clamp(min=1e-30))
        assert rel < (3e-2 if bf16 else 1e-4), (name, rel)
