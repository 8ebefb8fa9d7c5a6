"""north_star's own parity claim, end to end: one AdversarialVoxelNet training step (the loss and
every parameter gradient) on 6 full synthetic KITTI frames with fixed weights, HIP path in fp32
parity mode against the CPU oracle composition of the same step.

HIP (one GPU):   rpc_hard_voxelize -> fused perturber + compaction + HardSimpleVFE -> fp32
                 SparseEncoder -> fp32-MFMA SECOND / SECONDFPN (dense_f32.hip) -> fp32 head GEMM
                 -> rpc_anchor_head_loss -> AdversarialVoxelNet.loss combination -> parse_losses
                 -> backward through all of it
Oracle (host):   oracle/voxelize_ref.c -> the SAME plugin AdversarialVoxelNet.loss (pinned to the
                 reference's own adversarial_voxelnet.py:153-427 by the golden voxelnet_* fixtures)
                 on CPU modules: oracle perturber (float64, explicit compaction path of
                 adversarial_voxelnet.py:85-117, pinned by the golden perturber_* fixtures), HardSimpleVFE
                 formula, oracle SparseEncoder (fp32), torch-CPU fp32 SECOND / SECONDFPN with the same
                 weights, oracle Anchor3DHead targets + losses (float64) — each restating the
                 upstream module the reference calls (adversarial_voxelnet.py:135-145,168).

Tolerances (north_star: "voxel indices bit-exact, perturbed coords and detection losses within
1e-4 fp32"): voxels / coors / num_points bit-exact; perturbed point coordinates max |d| <= 1e-4;
every loss_* key and perturbation_l2_norm |d| <= 1e-4 * max(1, |ref|). Parameter gradients: the
gradient path crosses ~25 train-mode BatchNorm layers, whose batch statistics amplify fp32
summation-order differences — torch's own fp32 SECOND/FPN is 5-6e-3 (relative L2) from a float64
evaluation at this shape (tests/test_gpu_dense_bev.py::test_second_fpn_config_shape_fp32_engine_and_bf16_bounds),
so two correct fp32 evaluations (HIP, and the fp32 oracle whose dense part is torch fp32) differ by
up to ~1e-2 depending on how their rounding happens to correlate. The oracle composition is
therefore also run with float64 sparse encoder / SECOND / FPN, and each parameter gradient must be
(a) within relative L2 2e-2, cosine >= 0.9998 of the fp32 oracle and (b) within relative L2 1e-2 of
the float64 oracle, with the mean over all gradient tensors <= 2e-3 — as close to the exact step as
an fp32 evaluation of it gets (the fp32 oracle itself: mean 4.8e-3 / max 1.2e-2 for 3 classes,
2.3e-4 / 1.1e-3 for Car; HIP: 1.7e-3 / 5.7e-3 and 4.6e-4 / 2.6e-3, profiles/r02_e2e_parity_fp32.log).
"""
import copy

import numpy as np
import pytest
import torch
from torch import nn

import robustpointclouds_amd.plugin.models  # noqa: F401
from oracle import anchor_head as oh
from oracle import voxelize as ov
from oracle.perturber import OraclePerturber, perturb_voxels
from oracle.sparse_encoder import OracleSparseEncoder, implementation_masks
from robustpointclouds_amd import dense_bev
from robustpointclouds_amd.adversarial_loss import parse_losses
from robustpointclouds_amd.anchor_head import pack_gt
from robustpointclouds_amd.plugin.models.detectors.adversarial_voxelnet import AdversarialVoxelNet
from robustpointclouds_amd.synthetic import KITTI_PC_RANGE, KITTI_VOXEL_SIZE, kitti_batch
from robustpointclouds_amd.trainer import Trainer, make_kitti_model
from tests._dense_masks import FlipStats, engine_masks, follow_masks

pytestmark = pytest.mark.gpu
B = 6
LOSS_TOL = 1e-4
GRAD_REL = 2e-2
GRAD_F64_MAX = 1e-2
GRAD_F64_MEAN = 2e-3
FLIP_PRE_MAX = 1e-4   # a dense or sparse ReLU decision float64 makes differently lies within this of 0 (x channel max)
# Round 3 measured middle.11.gamma at 1.005e-2 from float64 and loosened this bound; round 4 re-ran the test with
# each backward variant switched off (tools/gpu_e2e_ab.sh: default, RPC_SPARSE_NATIVE=0, RPC_DENSE_BNFUSE=0, both;
# profiles/r04_e2e_backward_ab.log): all four give the same gradients — the one-call sparse backward is bit-identical
# to the layer loop and the fused BatchNorm-backward sums are a bf16-only path — with HIP 1.66e-3 mean / 4.84e-3
# max from float64 (middle.11.gamma well below 1e-2; the fp32 oracle itself 4.84e-3 / 1.21e-2). The fixed bound
# holds for every tensor again, with no exception.


class _VFE(nn.Module):            # upstream HardSimpleVFE formula (…3class.py:17)
    def forward(self, features, num_points, coors):
        return features[:, :, :4].sum(dim=1) / num_points.type_as(features).view(-1, 1)


class _Middle(nn.Module):
    """The oracle sparse encoder; with `masks`, evaluated on the HIP encoder's ReLU decisions."""

    def __init__(self, enc, dtype):
        super().__init__()
        self.enc, self.dtype = enc, dtype
        self.masks = None
        self.flips = None   # FlipStats: adopted sparse decisions that differ from this oracle's own

    def forward(self, feats, coors, batch_size):
        return self.enc.forward(feats.to(self.dtype), coors.numpy(), batch_size,
                                masks=self.masks, flips=self.flips).to(self.dtype)


class _Adversary(nn.Module):
    def __init__(self, op):
        super().__init__()
        self.op = op

    def forward(self, x):
        out, ld = self.op.forward(x)
        return out.to(x.dtype), ld


class _Head(nn.Module):
    """Anchor3DHead restatement: stacked 1x1 conv (float64) + oracle targets / losses, dict of lists."""

    def __init__(self, head, H, W):
        super().__init__()
        self.cfg = oh.cfg_of(head)
        w, b = head._stacked()
        self.w = nn.Parameter(w.detach().cpu().double().clone())
        self.b = nn.Parameter(b.detach().cpu().double().clone())
        g = head.prior_generator
        self.anchors = oh.grid_anchors(H, W, g.ranges, g.sizes, g.rotations)
        self.splits = [c.weight.shape[0] for c in head._convs()]

    def loss(self, x, samples):
        z = nn.functional.conv2d(x[0].double(), self.w)
        r = oh.head_losses_from_z(self.cfg, z, self.b, self.anchors, samples["gt_boxes"], samples["gt_labels"])
        return dict(loss_cls=[r["loss_cls"]], loss_bbox=[r["loss_bbox"]], loss_dir=[r["loss_dir"]])


def _perturber_weights(adv):
    lin = [m for m in adv.model if isinstance(m, nn.Linear)]
    bns = [m for m in adv.model if isinstance(m, nn.BatchNorm1d)]
    att = [m for m in adv.attention if isinstance(m, nn.Linear)]
    w = {}
    for l, m in enumerate(lin):
        w[f"W{l}"], w[f"b{l}"] = m.weight.detach().cpu().numpy(), m.bias.detach().cpu().numpy()
    for l, m in enumerate(bns):
        w[f"g{l}"], w[f"be{l}"] = m.weight.detach().cpu().numpy(), m.bias.detach().cpu().numpy()
    for l, m in enumerate(att):
        w[f"Wa{l}"], w[f"ba{l}"] = m.weight.detach().cpu().numpy(), m.bias.detach().cpu().numpy()
    return w, lin, bns, att


def _rel(a, b):
    a, b = a.double().flatten(), b.double().flatten()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


def _cos(a, b):
    a, b = a.double().flatten(), b.double().flatten()
    return float((a @ b) / (a.norm() * b.norm()).clamp_min(1e-30))


class _Oracle:
    """The oracle composition of the step at one dtype for the sparse encoder / SECOND / FPN (the
    perturber and head restatements are float64 in both)."""

    def __init__(self, model, hidden, w, dtype):
        self.dtype = dtype
        self.model = model
        self.enc = OracleSparseEncoder(model.middle_encoder, dtype=dtype)
        self.backbone = copy.deepcopy(model.backbone).cpu().to(dtype)
        self.neck = copy.deepcopy(model.neck).cpu().to(dtype)
        self.backbone.hip = self.neck.hip = False
        self.ref = AdversarialVoxelNet(adversary_cfg=dict(type="VoxelPerturber", hidden_channels=list(hidden)),
                                       regularization_weight=model.regularization_weight, voxel_encoder=_VFE(),
                                       middle_encoder=_Middle(self.enc, dtype), backbone=self.backbone,
                                       neck=self.neck, bbox_head=_Head(model.bbox_head, 200, 176))
        self.op = OraclePerturber(w, 4, hidden, dtype=torch.float64)
        self.ref.adversary = _Adversary(self.op)
        self.ref.train()
        self.ref._epoch = 3

    def step(self, rv, rn, rc, cb, cl, B, masks=None, dense_masks=None, flips=None, sparse_flips=None):
        """masks / dense_masks: the sparse encoder's / the dense engine's ReLU decisions (oracle/sparse_encoder.py,
        tests/_dense_masks.py); the decisions that differ from this oracle's own are counted in `flips` (dense) and
        `sparse_flips` (sparse)."""
        self.ref.middle_encoder.masks = masks
        self.ref.middle_encoder.flips = sparse_flips
        hooks = [] if dense_masks is None else follow_masks((self.model.backbone, self.model.neck),
                                                            (self.backbone, self.neck), dense_masks, flips)
        rbatch = dict(voxels=dict(voxels=torch.from_numpy(rv).to(self.dtype), num_points=torch.from_numpy(rn),
                                  coors=torch.from_numpy(rc)), batch_size=B)
        self.losses = self.ref.loss(rbatch, dict(gt_boxes=cb, gt_labels=cl))
        self.total, _ = parse_losses(self.losses)
        self.total.backward()
        for h in hooks:
            h.remove()

    def grads(self, nlin, natt, nbn):
        out = []
        g = self.op.grads()
        out += [g[f"dW{l}"] for l in range(nlin)] + [g[f"dWa{l}"] for l in range(natt)]
        out += [g[f"dg{l}"] for l in range(nbn)]
        for p in self.enc.params:
            out += [p["W"].grad, p["g"].grad]
        out += [p.grad for p in self.backbone.parameters()] + [p.grad for p in self.neck.parameters()]
        hw = torch.split(self.ref.bbox_head.w.grad, self.ref.bbox_head.splits)
        hb = torch.split(self.ref.bbox_head.b.grad, self.ref.bbox_head.splits)
        for gw, gbias in zip(hw, hb):
            out += [gw, gbias]
        return out


def _hip_grads(model):
    """(name, grad) in the order of _Oracle.grads()."""
    adv = model.adversary
    lin = [m for m in adv.model if isinstance(m, nn.Linear)]
    bns = [m for m in adv.model if isinstance(m, nn.BatchNorm1d)]
    att = [m for m in adv.attention if isinstance(m, nn.Linear)]
    out = [(f"adversary.W{l}", m.weight.grad) for l, m in enumerate(lin)]
    out += [(f"adversary.Wa{l}", m.weight.grad) for l, m in enumerate(att)]
    out += [(f"adversary.g{l}", m.weight.grad) for l, m in enumerate(bns)]
    for i, m in enumerate(model.middle_encoder.layers()):
        out += [(f"middle.{i}.W", m[0].weight.grad), (f"middle.{i}.gamma", m[1].weight.grad)]
    out += [(f"backbone.{n}", p.grad) for n, p in model.backbone.named_parameters()]
    out += [(f"neck.{n}", p.grad) for n, p in model.neck.named_parameters()]
    for c in model.bbox_head._convs():
        out += [("head.weight", c.weight.grad), ("head.bias", c.bias.grad)]
    return out


@pytest.mark.parametrize("classes", [3, 1])
def test_adversarial_step_fp32_hip_matches_oracle(classes):
    dev = torch.device("cuda")
    torch.manual_seed(11 + classes)
    model = make_kitti_model(num_classes=classes, device=dev, epoch=3)
    Trainer._select_engines(model, bf16=False)
    model.train()
    hidden = model.adversary.hidden_channels
    pts, boxes, labels = kitti_batch(B, seed0=500 + 10 * classes, num_classes=classes)

    # ---- oracle models (fp32 and float64), built from the GPU model's initial weights
    w = _perturber_weights(model.adversary)[0]
    o32 = _Oracle(model, hidden, w, torch.float32)
    o64 = _Oracle(model, hidden, w, torch.float64)

    # ---- HIP step (the sparse encoder's debug trace on: its ReLU decisions for the oracle, below)
    model.middle_encoder.debug = []
    dense_bev.DEBUG = []
    gpts = [torch.from_numpy(p).to(dev) for p in pts]
    batch = model.data_preprocessor(dict(inputs=dict(points=gpts)), training=True)["inputs"]
    batch["batch_size"] = B
    gb, gl = pack_gt(list(zip(boxes, labels)), dev)
    losses = model.loss(batch, dict(gt_boxes=gb, gt_labels=gl))
    total, log = parse_losses(losses)
    total.backward()
    torch.cuda.synchronize()

    # ---- voxelisation: bit-exact
    rv, rc, rn = ov.voxelize_frames(pts, KITTI_VOXEL_SIZE, KITTI_PC_RANGE, 5, 16000)
    vd = batch["voxels"]
    assert np.array_equal(vd["coors"].cpu().numpy(), rc)
    assert np.array_equal(vd["num_points"].cpu().numpy(), rn)
    assert np.array_equal(vd["voxels"].cpu().numpy().view(np.uint32), rv.view(np.uint32))

    # ---- perturbed coordinates (fused kernel's scattered voxels vs the oracle's explicit path)
    _, rpert, _ = perturb_voxels(OraclePerturber(w, 4, hidden, dtype=torch.float64), rv, rn)
    dp = (model._last_perturbed_voxels.cpu().double() - rpert).abs().max().item()
    assert dp <= 1e-4, dp

    # ---- oracle steps
    cb, cl = pack_gt(list(zip(boxes, labels)), torch.device("cpu"))
    # the sparse encoder's oracle on HIP's ReLU decisions (oracle/sparse_encoder.py `masks`): an fp32 pre-activation
    # within a rounding of 0 lands on either side, and one flipped decision moved gradients by up to 1e-2 (middle.8.gamma
    # 1.09e-2 vs the fp32 oracle's own 1.21e-2, gpurun_out r05j) — float64 arithmetic on the same branch instead
    masks = implementation_masks(model.middle_encoder.debug)
    model.middle_encoder.debug = None
    # likewise the dense SECOND / SECONDFPN on the engine's decisions (tests/_dense_masks.py; one flipped
    # decision moved backbone.blocks.1.1.bias by 1.04e-2 for Car, gpurun_out r05m)
    dmasks = engine_masks(dense_bev.DEBUG)
    dense_bev.DEBUG = None
    flips, sflips = FlipStats(), FlipStats()
    o32.step(rv, rn, rc, cb, cl, B, masks, dmasks)
    o64.step(rv, rn, rc, cb, cl, B, masks, dmasks, flips, sflips)
    print(f"dense ReLU decisions differing from float64's: {flips.flips} (max |pre| {flips.worst:.1e} of channel max)")
    print(f"sparse ReLU decisions differing from float64's: {sflips.flips} (max |act| {sflips.worst:.1e} of channel "
          f"max; per layer {sflips.per_layer})")
    assert flips.worst <= FLIP_PRE_MAX, flips.worst
    assert sflips.worst <= FLIP_PRE_MAX, sflips
    rlosses, rtotal = o32.losses, o32.total

    # ---- losses: every key within 1e-4 of the fp32 oracle
    assert set(losses) == set(rlosses), (sorted(losses), sorted(rlosses))
    report = {}
    for k in rlosses:
        a = losses[k][0] if isinstance(losses[k], (list, tuple)) else losses[k]
        r = rlosses[k][0] if isinstance(rlosses[k], (list, tuple)) else rlosses[k]
        a, r = float(a.detach()), float(r.detach())
        report[k] = (a, r)
        assert abs(a - r) <= LOSS_TOL * max(1.0, abs(r)), (k, a, r)
    assert abs(float(total) - float(rtotal)) <= LOSS_TOL * max(1.0, abs(float(rtotal)))
    print("losses (hip, oracle):", report)

    # ---- gradients: against the fp32 oracle, and no further from the float64 oracle than it is
    _, lin, bns, att = _perturber_weights(model.adversary)
    hg = _hip_grads(model)
    g32, g64 = o32.grads(len(lin), len(att), len(bns)), o64.grads(len(lin), len(att), len(bns))
    assert len(hg) == len(g32) == len(g64)
    worst = []
    for (name, a), r, r64 in zip(hg, g32, g64):
        assert a is not None and r is not None and r64 is not None, name
        a = a.cpu()
        rel, cos = _rel(a, r.cpu()), _cos(a, r.cpu())
        e_hip, e_ora = _rel(a, r64), _rel(r.cpu(), r64)
        worst.append((rel, name, cos, e_hip, e_ora))
    worst.sort(reverse=True)
    print("worst gradient rel-L2 (vs fp32 oracle, cos, hip vs f64, fp32 oracle vs f64):", worst[:6])
    ora_level = max(w[4] for w in worst)
    mean_hip = sum(w[3] for w in worst) / len(worst)
    mean_ora = sum(w[4] for w in worst) / len(worst)
    print(f"vs float64: hip mean {mean_hip:.2e} max {max(w[3] for w in worst):.2e}; "
          f"fp32 oracle mean {mean_ora:.2e} max {ora_level:.2e}")
    for rel, name, cos, e_hip, e_ora in worst:
        assert rel <= GRAD_REL and cos >= 0.9998, (name, rel, cos)
        # no farther from float64 than GRAD_F64_MAX, every tensor
        assert e_hip <= GRAD_F64_MAX, (name, e_hip, e_ora)
    assert mean_hip <= GRAD_F64_MEAN, (mean_hip, mean_ora)
