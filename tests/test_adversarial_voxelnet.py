"""a9/a10/a11 parity: AdversarialVoxelNet.loss (loss combination, epoch gate) + mmengine
parse_losses against the golden `voxelnet_*` fixtures, which were produced by running the
reference's own AdversarialVoxelNet (models/detectors/adversarial_voxelnet.py:153-427) with
stand-in VFE / middle / head modules (tests/golden/make_golden.py:233-305).

* CPU: the plugin detector with the CPU oracle perturber in the adversary slot (host logic of
  extract_feat's explicit compaction path, combine_adversarial_losses, parse_losses, gate).
* GPU: the plugin detector with its real HIP VoxelPerturber, both through the explicit path and
  through the fused HardSimpleVFE path (rpc_perturber_forward/backward with in-kernel compaction).
"""
import os

import numpy as np
import pytest
import torch
from torch import nn

import robustpointclouds_amd.plugin.models  # noqa: F401  (registers the plugin types)
from oracle.perturber import OraclePerturber
from robustpointclouds_amd.adversarial_loss import parse_losses
from robustpointclouds_amd.plugin.models.detectors.adversarial_voxelnet import AdversarialVoxelNet
from robustpointclouds_amd.voxelnet import HardSimpleVFE
from tests.conftest import GOLDEN

TAGS = ["list_e3", "list_e7", "tensor_e3", "gate_e2"]


class StandInVFE(nn.Module):          # make_golden.py:233-237 (HardSimpleVFE semantics)
    def forward(self, features, num_points, coors):
        return features[:, :, :4].sum(dim=1) / num_points.type_as(features).view(-1, 1)


class StandInMiddle(nn.Module):       # make_golden.py:240-244
    def forward(self, feats, coors, batch_size):
        out = feats.new_zeros(batch_size, feats.shape[1])
        return out.index_add(0, coors[:, 0].long(), feats.to(out.dtype))


class StandInHead(nn.Module):         # make_golden.py:247-259
    def __init__(self, w, listy):
        super().__init__()
        self.w = nn.Parameter(torch.from_numpy(np.asarray(w, np.float32)))
        self.listy = listy

    def loss(self, x, samples):
        y = (x.float() * 1e-2) @ self.w
        lc = (y[:, 0] ** 2).mean() * 1e-3 + 0.5
        lb = (y[:, 1].abs()).mean() * 1e-3 + 0.25
        ld = torch.sigmoid(y[:, 2]).mean() * 0.1
        if self.listy:
            return dict(loss_cls=[lc], loss_bbox=[lb], loss_dir=[ld])
        return dict(loss_cls=lc, loss_bbox=lb, loss_dir=ld)


class OracleAdversary(nn.Module):
    """Test-only: the CPU oracle perturber in the adversary slot (same (out, dict) contract)."""

    def __init__(self, d, hidden):
        super().__init__()
        self.op = OraclePerturber(d, 4, hidden)

    def forward(self, x):
        out, ld = self.op.forward(x)
        return out.to(x.dtype), ld


def _load(tag):
    return dict(np.load(os.path.join(GOLDEN, f"voxelnet_{tag}.npz")))


def _model(d, voxel_encoder, dev):
    hidden = [int(h) for h in d["hidden"]]
    m = AdversarialVoxelNet(adversary_cfg=dict(type="VoxelPerturber", hidden_channels=hidden),
                            regularization_weight=0.02, voxel_encoder=voxel_encoder,
                            middle_encoder=StandInMiddle(), backbone=nn.Identity(), neck=None,
                            bbox_head=StandInHead(d["head_w"], bool(d["listy"])))
    m = m.to(dev)
    m.train()
    m._epoch = int(d["epoch"])
    return m


def _inputs(d, dev):
    return {"voxels": {"voxels": torch.from_numpy(d["vox"]).to(dev),
                       "num_points": torch.from_numpy(d["num_points"]).to(dev),
                       "coors": torch.from_numpy(d["coors"]).to(dev)}}


def _check_losses(d, losses, total, tol):
    keys = [k[2:] for k in d if k.startswith("L_")]
    assert set(keys) == set(losses), (sorted(keys), sorted(losses))   # same key set as the reference
    for k in keys:
        v = losses[k]
        v = v[0] if isinstance(v, (list, tuple)) else v
        v = v.detach()
        assert abs(float(v) - float(d["L_" + k])) <= tol * max(1.0, abs(float(d["L_" + k]))), k
    assert abs(float(total) - float(d["total"])) <= tol * max(1.0, abs(float(d["total"])))


@pytest.mark.parametrize("tag", TAGS)
def test_loss_combination_matches_reference_cpu(tag):
    d = _load(tag)
    hidden = [int(h) for h in d["hidden"]]
    m = _model(d, StandInVFE(), torch.device("cpu"))
    m.adversary = OracleAdversary(d, hidden)
    losses = m.loss(_inputs(d, "cpu"), [None] * 2)
    total, log_vars = parse_losses(losses)
    _check_losses(d, losses, total, 1e-5)
    total.backward()
    g = m.adversary.op.grads()
    for l in range(6):
        np.testing.assert_allclose(g[f"dW{l}"].numpy(), d[f"dW{l}"], atol=2e-5 * max(1.0, np.abs(d[f"dW{l}"]).max()))
    for l in range(2):
        np.testing.assert_allclose(g[f"dWa{l}"].numpy(), d[f"dWa{l}"], atol=2e-5)
    np.testing.assert_allclose(m.bbox_head.w.grad.numpy(), d["dhead_w"], rtol=1e-4, atol=1e-7)
    if tag == "gate_e2":   # epoch < 3: adversary closed, zero adversarial terms, no grads into it
        assert all(float(losses[k]) == 0.0 for k in ("loss_adversarial", "loss_l2_regularization"))
        assert all(float(t.abs().max()) == 0.0 for t in g.values())


def _set_weights(adv, d):
    lin = [m for m in adv.model if isinstance(m, nn.Linear)]
    bns = [m for m in adv.model if isinstance(m, nn.BatchNorm1d)]
    att = [m for m in adv.attention if isinstance(m, nn.Linear)]
    with torch.no_grad():
        for l, m in enumerate(lin):
            m.weight.copy_(torch.from_numpy(d[f"W{l}"]))
            m.bias.copy_(torch.from_numpy(d[f"b{l}"]))
        for l, m in enumerate(bns):
            m.weight.copy_(torch.from_numpy(d[f"g{l}"]))
            m.bias.copy_(torch.from_numpy(d[f"be{l}"]))
        for l, m in enumerate(att):
            m.weight.copy_(torch.from_numpy(d[f"Wa{l}"]))
            m.bias.copy_(torch.from_numpy(d[f"ba{l}"]))
    return lin, att


@pytest.mark.gpu
@pytest.mark.parametrize("fused", [True, False])
@pytest.mark.parametrize("tag", TAGS)
def test_adversarial_voxelnet_hip_matches_reference(tag, fused):
    d = _load(tag)
    dev = torch.device("cuda")
    m = _model(d, HardSimpleVFE() if fused else StandInVFE(), dev)
    lin, att = _set_weights(m.adversary, d)
    losses = m.loss(_inputs(d, dev), [None] * 2)
    total, _ = parse_losses(losses)
    _check_losses(d, losses, total, 1e-4)
    total.backward()
    for l, mod in enumerate(lin):
        got = mod.weight.grad.cpu().numpy() if mod.weight.grad is not None else np.zeros_like(d[f"dW{l}"])
        np.testing.assert_allclose(got, d[f"dW{l}"], atol=1e-4 * max(1.0, np.abs(d[f"dW{l}"]).max()))
    for l, mod in enumerate(att):
        got = mod.weight.grad.cpu().numpy() if mod.weight.grad is not None else np.zeros_like(d[f"dWa{l}"])
        np.testing.assert_allclose(got, d[f"dWa{l}"], atol=1e-4)
    np.testing.assert_allclose(m.bbox_head.w.grad.cpu().numpy(), d["dhead_w"], rtol=1e-3, atol=1e-6)
