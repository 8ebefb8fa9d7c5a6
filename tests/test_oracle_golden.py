"""The perturber oracle (oracle/perturber.py) against golden vectors produced by running
the reference VoxelPerturber itself (tests/golden/make_golden.py)."""
import os

import numpy as np
import pytest
import torch

from oracle.perturber import OraclePerturber, perturb_voxels
from tests.conftest import GOLDEN

CASES = ["car_small", "car_clamp", "3class", "nus"]


def _load(tag):
    return dict(np.load(os.path.join(GOLDEN, f"perturber_{tag}.npz")))


@pytest.mark.parametrize("tag", CASES)
def test_oracle_forward_backward_matches_reference(tag):
    d = _load(tag)
    F = int(d["F"])
    op = OraclePerturber(d, F, d["hidden"], dtype=torch.float64)
    out, ld = op.forward(d["x"], training=True)
    np.testing.assert_allclose(out.detach().numpy(), d["out"], rtol=0, atol=2e-5)
    for k in ["l2_norm", "intensity_loss", "bias_loss", "imbalance_loss"]:
        np.testing.assert_allclose(ld[k].item(), float(d[k]), rtol=2e-5, atol=1e-7)
    c = d["c"].astype(np.float64)
    loss = (out * torch.from_numpy(d["G"].astype(np.float64))).sum() + c[0] * ld["l2_norm"] + \
        c[1] * ld["intensity_loss"] + c[2] * ld["bias_loss"] + c[3] * ld["imbalance_loss"]
    loss.backward()
    g = op.grads()
    for k, v in g.items():
        ref = d[k]
        scale = max(np.abs(ref).max(), 1e-3)
        tol = 1e-3
        if k[:2] == "db" and k[2:].isdigit() and int(k[2:]) < 5:
            # bias of a Linear feeding a train-mode BatchNorm: exact grad is 0, the fp32
            # reference holds cancellation noise of the order of its dW
            scale = max(scale, np.abs(d["dW" + k[2:]]).max())
            tol = 2e-3
        np.testing.assert_allclose(v.numpy(), ref, rtol=0, atol=tol * scale, err_msg=k)
    for l in range(5):
        np.testing.assert_allclose(op.rm[l].numpy(), d[f"rm{l}"], rtol=1e-5, atol=1e-5)
        np.testing.assert_allclose(op.rv[l].numpy(), d[f"rv{l}"], rtol=1e-4, atol=1e-5)
    # eval mode on the running stats updated by the train step
    oute, lde = op.forward(d["x_eval"], training=False)
    np.testing.assert_allclose(oute.detach().numpy(), d["out_eval"], rtol=0, atol=5e-5)
    np.testing.assert_allclose(lde["l2_norm"].item(), float(d["l2_norm_eval"]), rtol=5e-5)


def test_clamp_fixture_engages_grad_hook():
    d = _load("car_clamp")
    assert any(np.abs(d[k]).max() >= 0.1 - 1e-7 for k in d if k.startswith("dW"))


def test_fused_voxel_path_is_the_compaction_of_the_reference():
    """perturb_voxels() on a voxel tensor == perturber on the reference's valid-point set."""
    d = _load("car_small")
    rng = np.random.default_rng(0)
    V, P = 200, 5
    vox = np.zeros((V, P, 4), np.float32)
    npts = rng.integers(1, 6, V).astype(np.int32)
    for v in range(V):
        vox[v, :npts[v]] = d["x"][rng.integers(0, len(d["x"]), npts[v])]
    vox[3, 0] = [1.0, -1.0, 0.0, 0.0]           # real point with zero feature sum: not perturbed
    op = OraclePerturber(d, 4, d["hidden"])
    vfe, pert, ld = perturb_voxels(op, vox, npts)
    flat = vox.reshape(-1, 4)
    valid = flat.sum(1) != 0
    op2 = OraclePerturber(d, 4, d["hidden"])
    out2, ld2 = op2.forward(flat[valid])
    np.testing.assert_allclose(pert.detach().numpy().reshape(-1, 4)[valid], out2.detach().numpy(), atol=1e-12)
    assert np.array_equal(pert.detach().numpy()[3, 0], vox[3, 0])
    assert np.all(pert.detach().numpy().reshape(-1, 4)[~valid] == flat[~valid])
    ref_vfe = pert.detach().numpy()[:, :, :4].sum(1) / npts[:, None]
    np.testing.assert_allclose(vfe.detach().numpy(), ref_vfe, atol=1e-12)
