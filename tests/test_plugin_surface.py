"""(b) drop-in boundary: the reference's config-driven import surface and Runner entry points.

The reference's 3-class config loads the plugin through
`custom_imports=dict(imports=['models', 'models.detectors.adversarial_voxelnet', 'custom_hook',
'mmdet.models.losses'])` (…3class.py:9-11) with the plugin directory on sys.path, builds
`model=dict(type='AdversarialVoxelNet', ...)` (:14-120), the hooks (:123-126) and the optim
wrapper (:130-139), and mmengine's Runner then calls `model.train_step(data, optim_wrapper)`.
The config values come from tests/golden/config_*.json — extracted from the reference config files
as data by tests/golden/make_config_fixtures.py (no reference file is read at test time)."""
import json
import os
import subprocess
import sys

import pytest
import torch

from tests.conftest import GOLDEN, ROOT

PLUGIN = os.path.join(ROOT, "robustpointclouds_amd", "plugin")


def _cfg(tag):
    with open(os.path.join(GOLDEN, f"config_{tag}.json")) as f:
        return json.load(f)


_IMPORT_SURFACE = r'''
import importlib, json, sys
sys.path[:0] = [{root!r}, {plugin!r}]
cfg = json.load(open({cfg!r}))
imported, missing = [], []
for name in cfg["custom_imports"]["imports"]:
    if name.startswith("mmdet."):          # upstream mmdet: not installed in this image
        try:
            importlib.import_module(name)
        except ImportError:
            missing.append(name)
        continue
    importlib.import_module(name)
    imported.append(name)
import torch
from robustpointclouds_amd.registry import HOOKS, MODELS
model = MODELS.build(cfg["model"])
hooks = [HOOKS.build(h) for h in cfg.get("custom_hooks", [])]
adv = model.adversary
out = dict(imported=imported, missing=missing,
           model=type(model).__name__, model_module=type(model).__module__,
           adversary=type(adv).__name__, adversary_module=type(adv).__module__,
           perturber_params=sum(p.numel() for p in adv.parameters()),
           keys=sorted(k for k in model.state_dict() if k.startswith("adversary.")),
           hooks=[type(h).__name__ for h in hooks],
           nan_max=[getattr(h, "max_nan_count", None) for h in hooks],
           num_classes=model.bbox_head.num_classes, num_anchors=model.bbox_head.num_anchors,
           reg_w=model.regularization_weight, hidden=adv.hidden_channels,
           params=sum(p.numel() for p in model.parameters()))
print("RESULT" + json.dumps(out))
'''


def _run_surface(tag):
    code = _IMPORT_SURFACE.format(root=ROOT, plugin=PLUGIN, cfg=os.path.join(GOLDEN, f"config_{tag}.json"))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=600, cwd="/tmp")
    assert r.returncode == 0, r.stderr[-3000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("RESULT")][-1]
    return json.loads(line[len("RESULT"):])


def test_3class_config_import_surface_and_build():
    """custom_imports resolve from the plugin dir as top-level `models` / `custom_hook`, and the
    config's model / hooks dicts build through the registries (mmengine absent: the local ones)."""
    r = _run_surface("kitti3class")
    assert r["imported"] == ["models", "models.detectors.adversarial_voxelnet", "custom_hook"]
    assert r["missing"] == ["mmdet.models.losses"]
    assert r["model"] == "AdversarialVoxelNet" and r["model_module"] == "models.detectors.adversarial_voxelnet"
    assert r["adversary"] == "VoxelPerturber" and r["adversary_module"] == "models.adversarial.voxel_perturber"
    assert r["perturber_params"] == 34641            # eager build (SURVEY finding 2), hidden [64, 128, 64]
    assert r["hidden"] == [64, 128, 64]
    assert "adversary.model.0.weight" in r["keys"] and "adversary.model.15.bias" in r["keys"]
    assert "adversary.model.1.running_var" in r["keys"] and "adversary.attention.2.weight" in r["keys"]
    assert r["hooks"] == ["EpochTrackerHook", "NaNDetectionHook"] and r["nan_max"][1] == 10
    assert r["num_classes"] == 3 and r["num_anchors"] == 6
    assert r["reg_w"] == 0.02


def test_car_config_adversary_defaults():
    """The Car config's adversary_cfg is just type='VoxelPerturber' (defaults, …car.py:14-17)."""
    cfg = _cfg("kitti_car")
    assert cfg["custom_imports"]["imports"] == ["models.detectors.adversarial_voxelnet",
                                                "models.adversarial.voxel_perturber"]
    from robustpointclouds_amd.plugin.models.builder import build_adversary
    adv = build_adversary(cfg["model"]["adversary_cfg"])
    assert adv.hidden_channels == [8, 16, 32] and sum(p.numel() for p in adv.parameters()) == 1601


def test_nuscenes_config_adversary():
    cfg = _cfg("nuscenes")
    from robustpointclouds_amd.plugin.models.builder import build_adversary
    adv = build_adversary(cfg["model"]["adversary_cfg"])
    assert adv.in_features == 5 and sum(p.numel() for p in adv.parameters()) == 5780


def test_forward_modes_and_optim_wrapper_on_host():
    """mmengine BaseModel.forward(mode=) dispatch and the optim-wrapper builder (host form)."""
    from robustpointclouds_amd.base_model import DetectorBase
    from robustpointclouds_amd.trainer import build_optim_wrapper

    class Toy(DetectorBase):
        def __init__(self):
            super().__init__()
            self.adversary = torch.nn.Linear(2, 1)
            self.lin = torch.nn.Linear(2, 1)

        def loss(self, inputs, data_samples):
            return dict(loss_a=self.lin(inputs).mean(), loss_b=[self.adversary(inputs).mean()],
                        perturbation_l2_norm=torch.ones(()))

        def predict(self, inputs, data_samples):
            return "predicted"

        def _forward(self, inputs, data_samples=None):
            return "tensor"

    m = Toy()
    x = torch.randn(4, 2)
    assert m(x, None, mode="predict") == "predicted" and m(x) == "tensor"
    with pytest.raises(RuntimeError):
        m(x, mode="bogus")
    ow = build_optim_wrapper(m, _cfg("kitti3class")["optim_wrapper"])
    lrs = sorted(g["lr"] for g in ow.param_groups)
    assert lrs == [1e-4, 2e-4]                     # adversary lr_mult 2.0
    m.data_preprocessor = lambda data, training: data
    w0 = m.lin.weight.detach().clone()
    log = m.train_step(dict(inputs=x, data_samples=None), ow)
    assert set(log) == {"loss", "loss_a", "loss_b", "perturbation_l2_norm"}
    assert float(log["loss"]) == pytest.approx(float(log["loss_a"] + log["loss_b"]))
    assert not torch.equal(w0, m.lin.weight)


class _Boxes:
    def __init__(self, t):
        self.tensor = t


class _Instances:
    def __init__(self, b, l):
        self.bboxes_3d = _Boxes(b)
        self.labels_3d = l


class _Sample:
    """Duck-typed mmdet3d Det3DDataSample (gt_instances_3d.bboxes_3d.tensor / .labels_3d)."""

    def __init__(self, b, l):
        self.gt_instances_3d = _Instances(b, l)


def test_pack_gt_accepts_det3d_data_samples():
    from robustpointclouds_amd.anchor_head import pack_gt
    b0, l0 = torch.randn(3, 7), torch.tensor([0, 2, 1])
    b1, l1 = torch.randn(1, 9), torch.tensor([1])
    gb, gl = pack_gt([_Sample(b0, l0), _Sample(b1, l1)], torch.device("cpu"))
    rb, rl = pack_gt([(b0, l0), (b1[:, :7], l1)], torch.device("cpu"))
    assert torch.equal(gb, rb) and torch.equal(gl, rl)
    assert gb.shape == (2, 3, 7) and gl[1].tolist() == [1, -1, -1]


@pytest.mark.gpu
@pytest.mark.parametrize("bf16", [True, False])
def test_runner_train_step_matches_trainer_bit_for_bit(bf16):
    """mmengine flow — model.train_step(dict(inputs=dict(points=<host tensors>), data_samples=
    <Det3DDataSamples>), optim_wrapper built from the config's optim_wrapper dict) — against the
    build's Trainer.train_step on the same frames: identical losses and parameters, bit for bit."""
    from robustpointclouds_amd.synthetic import kitti_batch
    from robustpointclouds_amd.trainer import Trainer, build_model, build_optim_wrapper
    from robustpointclouds_amd.voxelnet import second_kitti_cfg
    import robustpointclouds_amd.plugin.models  # noqa: F401
    dev = torch.device("cuda")
    cfg = _cfg("kitti3class")
    torch.manual_seed(5)
    a = build_model(cfg["model"]).to(dev)
    b = build_model(cfg["model"]).to(dev)
    b.load_state_dict(a.state_dict())
    a._epoch = b._epoch = 3
    s0 = {k: v.detach().clone() for k, v in a.state_dict().items()}
    pts, boxes, labels = kitti_batch(6, seed0=77, num_classes=3)
    # the build's trainer (padded GT dict, points already on the device)
    tr = Trainer(a, bf16=bf16, device=dev)
    for g in tr.opt.param_groups:
        g["lr"] = g["initial_lr"]                # undo the LinearLR start factor: the wrapper has no schedule
    from robustpointclouds_amd.anchor_head import pack_gt
    gb, gl = pack_gt(list(zip(boxes, labels)), dev)
    log_a = tr.train_step([torch.from_numpy(p).to(dev) for p in pts], dict(gt_boxes=gb, gt_labels=gl))
    # the reference Runner's call: host points + data samples, optim wrapper from the config dict
    ocfg = dict(cfg["optim_wrapper"])
    if bf16:
        ocfg.update(type="AmpOptimWrapper", dtype="bfloat16")
    b.train()
    ow = build_optim_wrapper(b, ocfg)
    data = dict(inputs=dict(points=[torch.from_numpy(p) for p in pts]),
                data_samples=[_Sample(torch.from_numpy(x), torch.from_numpy(y)) for x, y in zip(boxes, labels)])
    log_b = b.train_step(data, ow)
    torch.cuda.synchronize()
    assert set(log_a) == set(log_b)
    for k in log_a:
        assert torch.equal(log_a[k].detach().float().cpu(), log_b[k].detach().float().cpu()), k
    sa, sb = a.state_dict(), b.state_dict()
    for k in sa:
        assert torch.equal(sa[k], sb[k]), k
    for k in ("backbone.blocks.0.0.weight", "adversary.model.0.weight", "bbox_head.conv_cls.weight"):
        assert not torch.equal(sa[k], s0[k]), k
    assert b.__dict__["_engine_mode"] == bf16 and b.backbone.hip and b.neck.hip
