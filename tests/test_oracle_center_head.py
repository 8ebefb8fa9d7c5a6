"""§8(f3): known-answer checks of the CenterHead oracle restatement (CPU).

Parity w.r.t. upstream mmdet3d is unpinned (not vendored, see oracle/center_head.py); these pin the
restatement's own invariants: the gaussian peak is exactly 1 at the centre cell and symmetric,
gaussian_radius of a known box, the task slot order (class order within a task, then GT order),
the anno box encoding, and the focal / L1 loss values on hand-built inputs."""
import math

import torch

from oracle import center_head as oc
from tests._center_data import nus_gts


def test_gaussian_peak_and_symmetry():
    hm = torch.zeros(20, 20)
    oc.draw_heatmap_gaussian(hm, torch.tensor([7, 9], dtype=torch.int32), 3)
    assert hm[9, 7] == 1.0
    assert torch.equal(hm[9, 4:11], hm[9, 4:11].flip(0))
    assert torch.equal(hm[6:13, 7], hm[6:13, 7].flip(0))
    assert hm[9, 3] == 0.0 and hm[9, 11] == 0.0          # outside the 7x7 window
    sigma = 7 / 6
    assert float(hm[9, 8]) == float(torch.tensor(math.exp(-1 / (2 * sigma * sigma)), dtype=torch.float32))


def test_gaussian_radius_known_box():
    # a 4.5 m x 1.9 m car at 0.1 m voxels / 8 -> 5.625 x 2.375 cells
    r = oc.gaussian_radius((torch.tensor(4.5 / 0.8), torch.tensor(1.9 / 0.8)), 0.1)
    h, w, mo = 4.5 / 0.8, 1.9 / 0.8, 0.1
    b3, c3 = -2 * mo * (h + w), (mo - 1) * w * h
    r3 = (b3 + math.sqrt(b3 ** 2 - 4 * (4 * mo) * c3)) / 2
    assert abs(float(r) - r3) < 1e-5 and int(r) == 1       # -> max(min_radius=2, 1) = 2


def test_targets_slots_and_anno():
    cfg = oc.CenterCfg()
    boxes = torch.tensor([[10.0, 5.0, -1.0, 2.0, 4.0, 1.5, 0.3, 1.0, -2.0],     # truck (1) -> task 1 slot 0
                          [-20.0, 7.0, -1.2, 1.9, 4.5, 1.6, -0.2, 0.5, 0.0],    # car (0) -> task 0 slot 0
                          [0.0, 0.0, -1.0, 3.0, 8.0, 3.0, 1.0, 0.0, 0.0],       # construction_vehicle (2) -> task 1 slot 2
                          [30.0, -30.0, -1.0, 2.5, 6.0, 2.5, 0.0, 0.0, 0.0]])   # truck (1) -> task 1 slot 1
    labels = torch.tensor([1, 0, 2, 1])
    hms, annos, inds, masks = oc.targets_single(cfg, boxes, labels)
    # task 1 = (truck, construction_vehicle): trucks first in GT order (rows 0, 3), then row 2
    assert masks[1][:3].tolist() == [1, 1, 1] and masks[1][3] == 0
    cx, cy = int((10.0 + 51.2) / 0.1 / 8), int((5.0 + 51.2) / 0.1 / 8)
    assert int(inds[1][0]) == cy * 128 + cx
    a = annos[1][0]
    assert abs(float(a[2]) - (-1.0 + 0.75)) < 1e-6                      # gravity-centre z
    assert abs(float(a[3]) - math.log(2.0)) < 1e-6 and abs(float(a[6]) - math.sin(0.3)) < 1e-6
    assert float(hms[0][0].max()) == 1.0 and int(hms[1].eq(1).sum()) == 3


def test_losses_finite_and_edge_cases():
    cfg = oc.CenterCfg()
    g = torch.Generator().manual_seed(0)
    gts = nus_gts(2, seed=3)
    hm = [torch.randn(2, n, 128, 128, generator=g) for n in cfg.ncls]
    bx = [torch.randn(2, 10, 128, 128, generator=g) for _ in cfg.ncls]
    out = oc.losses(cfg, hm, bx, [b for b, _ in gts], [l for _, l in gts])
    assert len(out) == 12 and all(torch.isfinite(v) for v in out.values())
    # no objects at all: focal / max(0, 1), L1 = 0
    out0 = oc.losses(cfg, hm, bx, [torch.zeros(0, 9)] * 2, [torch.zeros(0, dtype=torch.long)] * 2)
    assert all(float(out0[f"task{t}.loss_bbox"]) == 0.0 for t in range(6))
