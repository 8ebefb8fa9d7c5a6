"""BASELINE config 4's parity: one AdversarialCenterPoint training step (every loss and every parameter
gradient) on synthetic nuScenes-like frames with fixed weights, HIP path in fp32 parity mode against the
CPU oracle composition of the same step (the SECOND counterpart is tests/test_gpu_e2e_parity.py).

HIP (one GPU):   rpc_hard_voxelize (F = 5) -> fused perturber + compaction + HardSimpleVFE -> fp32
                 basicblock SparseEncoder (128-wide fp32 convs) -> fp32-MFMA SECOND / SECONDFPN -> fp32
                 CenterHead (dense engine, rpc_dcn_*_f32, fp32 head images) -> rpc_center_head_loss ->
                 AdversarialCenterPoint.loss_by_feat_single combination -> parse_losses -> backward
Oracle (host):   oracle/voxelize_ref.c -> the SAME plugin AdversarialCenterPoint (whose combination the
                 golden centerpoint_* fixtures pin to models/detectors/adversarial_centerpoint.py:203-257)
                 on CPU modules: oracle perturber (float64, the explicit compaction path :77-81), the
                 HardSimpleVFE formula, oracle SparseEncoder, torch-CPU SECOND / SECONDFPN, the CenterHead
                 layer stack in torch with oracle/dcn.py, oracle/center_head.py targets + losses.

Tolerances: voxels bit-exact; every loss key within 1e-4 * max(1, |ref|) of the fp32 oracle (north_star); every
parameter gradient within GRAD_F64_MAX relative L2 of float64, their mean within GRAD_F64_MEAN, cosine >= COS_MIN
(the fixed bounds of tests/test_gpu_e2e_parity.py). Both oracles evaluate the sparse encoder and the dense
SECOND / SECONDFPN on HIP's ReLU decisions (same-branch parity: oracle/sparse_encoder.py `masks`,
tests/_dense_masks.py), and every dense or sparse decision the float64 oracle would take differently must lie
within FLIP_PRE_MAX of zero (r06: the sparse decisions are bounded too). r05 (gpurun_out r05o): 43 / 115 such decisions, all within 3.6e-6 of the channel's max
|pre|; HIP 4.7e-5 / 2.8e-4 mean, 1.2e-3 / 2.1e-3 max from float64 (fp32 oracle 3.8e-4 / 2.6e-4 mean) for
B = 2 one-sweep / B = 4 three-sweep frames. Without the dense masks one decision at x_hat ~ 0 with a large
gradient behind it moved the CenterPoint backbone's gradients by 1.3e-2 (tools/dbg_cp_bb.py: blocks.1.7.bias
6.3e-3 while blocks.1.7.weight stayed at 5.8e-5).

DCN offsets (r05). The DCN offset gradient is piecewise constant in the sampling position: it jumps where a
sample crosses a bilinear cell edge. With the offsets of r04's test (conv_offset weights N(0, 0.02), biases
U(-0.5, 0.5): positions spread over whole cells) ~12 of each DCN's 590k samples lie within 1e-5 of an edge, and
a 1e-5 relative change of the neck output (fp32 rounding: HIP 1.1e-5, torch fp32 4e-6) moves 1-3 of them across
(tools/archive/dbg_cp_flip.py, gpurun_out r05b). One crossing near a GT peak moved that DCN's offset-conv gradient by
2.3e-2 and, through the shared conv, every gradient upstream by ~1e-2 — for HIP and equally for the float64 oracle
fed HIP's neck output (tools/dbg_cp_sub.py: f64 | N_hip mean 5.5e-3), while HIP fed the float64 neck output was
1.4e-4 (mean) / 2.0e-3 (max) from float64. The test therefore draws offsets that keep every sampling position
mid-cell — conv_offset biases U(0.35, 0.65) and weights N(0, 5e-4) (the shared-conv features reach ~10 near
objects, so the offset conv adds up to ~0.1: positions n + 0.5 +- 0.25) — so the bilinear weights, their offset
gradients and the offset convs all stay active while no fp32 rounding can cross an edge. (With weights N(0, 0.004)
the offsets near objects still reached cell edges: the fp32 oracle itself was then 1.6e-3 mean / 2e-2 max from
float64, gpurun_out r05c.)
"""
import copy

import numpy as np
import pytest
import torch
import torch.nn.functional as Fn
from torch import nn

import robustpointclouds_amd.plugin.models  # noqa: F401
from oracle import center_head as och
from oracle import voxelize as ov
from oracle.dcn import deform_conv2d
from oracle.perturber import OraclePerturber
from oracle.sparse_encoder import OracleSparseEncoder, implementation_masks
from robustpointclouds_amd import dense_bev
from robustpointclouds_amd.adversarial_loss import parse_losses
from robustpointclouds_amd.center_head import _BOX_ORDER, pack_gt
from robustpointclouds_amd.centerpoint import NUS_PC_RANGE, NUS_VOXEL_SIZE
from robustpointclouds_amd.plugin.models.detectors.adversarial_centerpoint import AdversarialCenterPoint
from robustpointclouds_amd.synthetic import nus_frame, nus_gt_boxes
from tests._dense_masks import FlipStats, engine_masks, follow_masks

LOSS_TOL = 1e-4
GRAD_F64_MAX = 1e-2
GRAD_F64_MEAN = 2e-3
COS_MIN = 0.9995
FLIP_PRE_MAX = 1e-4   # a decision the float64 oracle makes differently lies within this of 0 (x channel max |pre|)


def init_mid_cell_offsets(model):
    """DCN offsets that keep every sampling position mid-cell (module docstring); upstream zero-initialises
    the offset convs, which would put every sample exactly ON a cell edge."""
    with torch.no_grad():
        for th in model.pts_bbox_head.task_heads:
            for dcn in (th.feature_adapt_cls, th.feature_adapt_reg):
                dcn.conv_offset.weight.normal_(0, 5e-4)
                dcn.conv_offset.bias.uniform_(0.35, 0.65)


class _VFE(nn.Module):            # upstream HardSimpleVFE(num_features=5) formula
    def forward(self, features, num_points, coors):
        return features[:, :, :5].sum(dim=1) / num_points.type_as(features).view(-1, 1)


class _Middle(nn.Module):
    """The oracle sparse encoder (with `masks`: on the HIP encoder's ReLU decisions); `out` keeps the last output."""

    def __init__(self, enc, dtype):
        super().__init__()
        self.enc, self.dtype = enc, dtype
        self.out = None
        self.masks = None
        self.flips = None   # FlipStats: adopted sparse decisions that differ from this oracle's own

    def forward(self, feats, coors, batch_size):
        out = self.enc.forward(feats.to(self.dtype), coors.numpy(), batch_size, masks=self.masks,
                               flips=self.flips).to(self.dtype)
        self.out = out.detach()
        return out


class _Adversary(nn.Module):
    def __init__(self, op):
        super().__init__()
        self.op = op

    def forward(self, x):
        out, ld = self.op.forward(x)
        return out.to(x.dtype), ld


class _CenterHead(nn.Module):
    """The CenterHead layer stack (shared ConvModule, per task two DCNSeparateHead DeformConv2dPacks with
    their offset convs, cls / reg ConvModule + final conv) in torch ops on a CPU copy of the module's
    parameters, train-mode BatchNorm, oracle/dcn.py; loss_by_feat = oracle/center_head.py losses."""

    def __init__(self, head, dtype):
        super().__init__()
        self.m = copy.deepcopy(head).cpu().to(dtype)
        self.cfg = och.CenterCfg()

    @staticmethod
    def _cm(cm, h):
        z = Fn.conv2d(h, cm.conv.weight, padding=1)
        m = z.mean((0, 2, 3), keepdim=True)
        v = z.var((0, 2, 3), unbiased=False, keepdim=True)
        return torch.relu((z - m) / torch.sqrt(v + cm.bn.eps) * cm.bn.weight.view(1, -1, 1, 1)
                          + cm.bn.bias.view(1, -1, 1, 1))

    def forward(self, feats):
        x = feats[0] if isinstance(feats, (list, tuple)) else feats
        y0 = self._cm(self.m.shared_conv, x)
        hms, boxes = [], []
        for th in self.m.task_heads:
            f = {}
            for br, dcn in (("cls", th.feature_adapt_cls), ("reg", th.feature_adapt_reg)):
                off = Fn.conv2d(y0, dcn.conv_offset.weight, dcn.conv_offset.bias, padding=1)
                f[br] = deform_conv2d(y0, off, dcn.weight, groups=4)
            fc = th.cls_head[1]
            hms.append(Fn.conv2d(self._cm(th.cls_head[0], f["cls"]), fc.weight, fc.bias, padding=1))
            parts = []
            for name in _BOX_ORDER:
                seq = getattr(th.task_head, name)
                parts.append(Fn.conv2d(self._cm(seq[0], f["reg"]), seq[1].weight, seq[1].bias, padding=1))
            boxes.append(torch.cat(parts, 1))
        return hms, boxes

    def loss_by_feat(self, outs, gts):
        hms, boxes = outs
        return dict(och.losses(self.cfg, hms, boxes, gts["boxes"], gts["labels"]))


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


class OracleStep:
    """The oracle composition of the step; the sparse encoder / SECOND / FPN / head stack in `dtype`, the
    perturber restatement in float64."""

    def __init__(self, model, dtype):
        self.model = model
        adv = model.adversary
        self.hidden = list(adv.hidden_channels)
        w, self.lin, self.bns, self.att = _perturber_weights(adv)
        self.enc = OracleSparseEncoder(model.pts_middle_encoder, dtype=dtype)
        backbone = copy.deepcopy(model.pts_backbone).cpu().to(dtype)
        neck = copy.deepcopy(model.pts_neck).cpu().to(dtype)
        backbone.hip = neck.hip = False
        self.ref = AdversarialCenterPoint(
            adversary_cfg=dict(type="VoxelPerturber", hidden_channels=self.hidden, sensor_error_bound=0.2,
                               voxel_size=NUS_VOXEL_SIZE, use_spatial_attention=True),
            adversarial_loss_weight=model.adversarial_loss_weight,
            regularization_weight=model.regularization_weight, pts_voxel_encoder=_VFE(),
            pts_middle_encoder=_Middle(self.enc, dtype), pts_backbone=backbone, pts_neck=neck,
            pts_bbox_head=_CenterHead(model.pts_bbox_head, dtype))
        self.op = OraclePerturber(w, 5, self.hidden, dtype=torch.float64)
        self.ref.adversary = _Adversary(self.op)
        self.ref.train()
        self.ref._epoch = model._epoch

    def step(self, rv, rn, rc, gts, masks=None, dense_masks=None, flips=None, sparse_flips=None):
        """masks: the sparse encoder's ReLU decisions (oracle/sparse_encoder.py), whose decisions that differ from
        this oracle's own are counted in `sparse_flips`; dense_masks: the dense engine's (tests/_dense_masks.py) for
        SECOND + SECONDFPN, counted in `flips`."""
        self.ref.pts_middle_encoder.masks = masks
        self.ref.pts_middle_encoder.flips = sparse_flips
        hooks = [] if dense_masks is None else follow_masks(
            (self.model.pts_backbone, self.model.pts_neck), (self.ref.pts_backbone, self.ref.pts_neck), dense_masks,
            flips)
        batch = dict(voxels=dict(voxels=torch.from_numpy(rv).to(self.enc.dtype), num_points=torch.from_numpy(rn),
                                 coors=torch.from_numpy(rc)), batch_size=len(gts["boxes"]))
        self.losses = self.ref.loss(batch, gts)
        self.total, _ = parse_losses(self.losses)
        print(f"  {self.enc.dtype} oracle forward done; backward ...", flush=True)
        self.total.backward()
        for h in hooks:
            h.remove()

    def grads(self):
        g = self.op.grads()
        out = [(f"adversary.W{l}", g[f"dW{l}"]) for l in range(len(self.lin))]
        out += [(f"adversary.Wa{l}", g[f"dWa{l}"]) for l in range(len(self.att))]
        out += [(f"adversary.g{l}", g[f"dg{l}"]) for l in range(len(self.bns))]
        for i, p in enumerate(self.enc.params):
            out += [(f"middle.{i}.W", p["W"].grad), (f"middle.{i}.gamma", p["g"].grad),
                    (f"middle.{i}.beta", p["b"].grad)]
        r = self.ref
        out += [(f"backbone.{n}", p.grad) for n, p in r.pts_backbone.named_parameters()]
        out += [(f"neck.{n}", p.grad) for n, p in r.pts_neck.named_parameters()]
        out += [(f"head.{n}", p.grad) for n, p in r.pts_bbox_head.m.named_parameters()]
        return out


def hip_grads(model):
    """(name, grad) in the order of OracleStep.grads()."""
    adv = model.adversary
    lin = [m for m in adv.model if isinstance(m, nn.Linear)]
    bns = [m for m in adv.model if isinstance(m, nn.BatchNorm1d)]
    att = [m for m in adv.attention if isinstance(m, nn.Linear)]
    out = [(f"adversary.W{l}", m.weight.grad) for l, m in enumerate(lin)]
    out += [(f"adversary.Wa{l}", m.weight.grad) for l, m in enumerate(att)]
    out += [(f"adversary.g{l}", m.weight.grad) for l, m in enumerate(bns)]
    for i, m in enumerate(model.pts_middle_encoder.layers()):
        out += [(f"middle.{i}.W", m[0].weight.grad), (f"middle.{i}.gamma", m[1].weight.grad),
                (f"middle.{i}.beta", m[1].bias.grad)]
    out += [(f"backbone.{n}", p.grad) for n, p in model.pts_backbone.named_parameters()]
    out += [(f"neck.{n}", p.grad) for n, p in model.pts_neck.named_parameters()]
    out += [(f"head.{n}", p.grad) for n, p in model.pts_bbox_head.named_parameters()]
    return out


def frames(seed0=900, B=2, sweeps=1):
    pts = [nus_frame(seed0 + i, sweeps=sweeps) for i in range(B)]
    gts = [nus_gt_boxes(seed0 + i) for i in range(B)]
    return pts, gts


def oracle_voxels(pts):
    return ov.voxelize_frames(pts, NUS_VOXEL_SIZE, NUS_PC_RANGE, 10, 90000)


@pytest.mark.gpu
@pytest.mark.timeout(600)
@pytest.mark.parametrize("B,sweeps", [(2, 1), (4, 10)])
def test_adversarial_centerpoint_step_fp32_hip_matches_oracle(B, sweeps):
    """r04's B = 2 one-sweep frames, and config 4 at its own size: B = 4 ten-sweep frames (360k voxels, the
    max_voxels cap; ~3 min with the float64 oracle step, profiles/r05_e2e_parity_cp_10sweeps.log — HIP 3.4e-4
    worst / 3.2e-5 mean from float64, the fp32 oracle 1.0e-3 / 9.9e-5), on the config's full grid
    (41 x 1024 x 1024 -> 128 x 128 BEV). The oracle's sparse encoder runs on HIP's ReLU decisions (oracle/sparse_encoder.py `masks`): 21 layers of
    ~10^6 fp32 pre-activations each put a few within a rounding of 0, and which side one lands on moved every
    gradient upstream by up to ~1e-2 — for torch fp32 against float64 as for HIP (fp32 oracle 2.3e-3 mean from
    float64 at B = 4, gpurun_out r05d)."""
    from robustpointclouds_amd.trainer import Trainer, make_nus_model
    dev = torch.device("cuda")
    torch.manual_seed(21)
    model = make_nus_model(device=dev, epoch=3)
    init_mid_cell_offsets(model)
    Trainer._select_engines(model, bf16=False)
    model.train()
    pts, gts = frames(B=B, sweeps=sweeps)
    o32 = OracleStep(model, torch.float32)
    o64 = OracleStep(model, torch.float64)
    rv, rc, rn = oracle_voxels(pts)
    ogts = dict(boxes=[torch.from_numpy(b) for b, _ in gts], labels=[torch.from_numpy(l) for _, l in gts])
    mid = {}
    model.pts_middle_encoder.register_forward_hook(lambda m, i, o: mid.__setitem__("hip", o.detach()))

    # ---- HIP step (the sparse encoder's and the dense engine's debug traces on: their ReLU decisions)
    model.pts_middle_encoder.debug = []
    dense_bev.DEBUG = []
    gpts = [torch.from_numpy(p).to(dev) for p in pts]
    batch = model.data_preprocessor(dict(inputs=dict(points=gpts)), training=True)["inputs"]
    batch["batch_size"] = B
    gb, gl = pack_gt([torch.from_numpy(b) for b, _ in gts], [torch.from_numpy(l) for _, l in gts], dev)
    losses = model.loss(batch, dict(gt_boxes=gb, gt_labels=gl))
    total, _ = parse_losses(losses)
    total.backward()
    torch.cuda.synchronize()
    masks = implementation_masks(model.pts_middle_encoder.debug)
    model.pts_middle_encoder.debug = None
    dmasks = engine_masks(dense_bev.DEBUG)
    dense_bev.DEBUG = None

    # ---- voxelisation: bit-exact
    vd = batch["voxels"]
    assert np.array_equal(vd["coors"].cpu().numpy(), rc)
    assert np.array_equal(vd["num_points"].cpu().numpy(), rn)
    assert np.array_equal(vd["voxels"].cpu().numpy().view(np.uint32), rv.view(np.uint32))

    # ---- oracle steps
    flips, sflips = FlipStats(), FlipStats()
    print(f"HIP step done ({rv.shape[0]} voxels); fp32 oracle step ...", flush=True)
    o32.step(rv, rn, rc, ogts, masks, dmasks)
    print("fp32 oracle step done; float64 oracle step ...", flush=True)
    o64.step(rv, rn, rc, ogts, masks, dmasks, flips, sflips)
    print(f"dense ReLU decisions differing from float64's: {flips.flips} (max |pre| {flips.worst:.1e} of channel max)")
    print(f"sparse ReLU decisions differing from float64's: {sflips.flips} (max |act| {sflips.worst:.1e} of channel "
          f"max; per layer {sflips.per_layer})")
    assert flips.worst <= FLIP_PRE_MAX, flips.worst
    assert sflips.worst <= FLIP_PRE_MAX, sflips
    eps_mid = _rel(mid["hip"].float().cpu(), o64.ref.pts_middle_encoder.out)
    print(f"B={B} sweeps={sweeps} voxels {rv.shape[0]}; encoder output: HIP vs float64 {eps_mid:.2e} "
          f"(fp32 oracle {_rel(o32.ref.pts_middle_encoder.out, o64.ref.pts_middle_encoder.out):.2e})")

    # ---- losses
    assert set(losses) == set(o32.losses), (sorted(losses), sorted(o32.losses))
    report = {}
    for k, r in o32.losses.items():
        a, r = float(losses[k].detach()), float(r.detach())
        report[k] = (a, r)
        assert abs(a - r) <= LOSS_TOL * max(1.0, abs(r)), (k, a, r)
    assert abs(float(total) - float(o32.total)) <= LOSS_TOL * max(1.0, abs(float(o32.total)))
    print("losses (hip, oracle):", report)

    # ---- gradients against float64, fixed bounds
    hg, g32, g64 = hip_grads(model), o32.grads(), o64.grads()
    assert [n for n, _ in hg] == [n for n, _ in g32] == [n for n, _ in g64]
    rows = []
    for (name, a), (_, r), (_, r64) in zip(hg, g32, g64):
        assert a is not None and r is not None and r64 is not None, name
        a = a.cpu()
        rows.append((_rel(a, r64), name, _cos(a, r64), _rel(r, r64)))
    rows.sort(reverse=True)
    print("gradient rel-L2 vs float64 (hip, cos, fp32 oracle), worst first:")
    for e, name, cos, e_ora in rows[:40]:
        print(f"  {name:48s} {e:.3e} {cos:.6f} {e_ora:.3e}")
    mean_hip = sum(r[0] for r in rows) / len(rows)
    mean_ora = sum(r[3] for r in rows) / len(rows)
    print(f"mean: hip {mean_hip:.2e}  fp32 oracle {mean_ora:.2e}")
    for e, name, cos, e_ora in rows:
        assert e <= GRAD_F64_MAX, (name, e)
        if e > 0:    # (a gradient that is exactly zero on both sides has no direction)
            assert cos >= COS_MIN, (name, cos)
    assert mean_hip <= GRAD_F64_MEAN, mean_hip
