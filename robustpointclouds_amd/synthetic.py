"""Seeded synthetic KITTI-shaped LiDAR frames and GT boxes.

There is no network on either box, so every test, the bench and the CPU baseline
run on frames produced here:

* HDL-64E-like rays: 64 beams, elevation -24.8°..+2°, azimuth ±45° in 0.17° steps,
  keep-probability 0.6 (≈20k raw points per frame);
* flat ground at z = -1.73 m (sensor at the origin), 15 % of rays return from an
  "object" at U(5, 60) m, the rest from a background wall at U(30, 110) m;
* N(0, 0.02) xyz jitter, intensity U[0, 1);
* GT: 6–10 boxes per frame with the anchor sizes of the KITTI configs
  (`configs/adversarial/adversarial-second_hv_secfpn_8xb6-80e_kitti-3d-3class.py:51`),
  yaw U(-π, π), bottom-centre z on the ground, inside the point-cloud range.

Frames are float32 `[N, 4]` (x, y, z, intensity) exactly like a KITTI `.bin`
(`configs/_base_/kitti-3d-car.py:46`, load_dim=4).
"""
from __future__ import annotations

import numpy as np

KITTI_PC_RANGE = (0.0, -40.0, -3.0, 70.4, 40.0, 1.0)
KITTI_VOXEL_SIZE = (0.05, 0.05, 0.1)
# Car / Pedestrian / Cyclist anchor sizes (dx, dy, dz), 3-class config :51
KITTI_SIZES = ((3.9, 1.6, 1.56), (0.8, 0.6, 1.73), (1.76, 0.6, 1.73))


def kitti_frame(seed: int, keep: float = 0.6) -> np.ndarray:
    """One HDL-64E-like frame, float32 [N, 4]."""
    rng = np.random.default_rng(seed)
    elev = np.deg2rad(np.linspace(-24.8, 2.0, 64))
    azim = np.deg2rad(np.arange(-45.0, 45.0, 0.17))
    el, az = np.meshgrid(elev, azim, indexing="ij")
    el = el.ravel()
    az = az.ravel()
    m = rng.random(el.shape[0]) < keep
    el, az = el[m], az[m]
    n = el.shape[0]
    r = rng.uniform(30.0, 110.0, n)                      # background wall
    down = el < 0
    r_ground = np.where(down, 1.73 / np.tan(np.maximum(-el, 1e-6)), np.inf)
    ground = down & (r_ground < 110.0)
    r = np.where(ground, r_ground, r)
    obj = rng.random(n) < 0.15
    r_obj = rng.uniform(5.0, 60.0, n)
    r = np.where(obj, np.minimum(r_obj, r), r)
    x = r * np.cos(el) * np.cos(az)
    y = r * np.cos(el) * np.sin(az)
    z = r * np.sin(el)
    z = np.where(ground & ~obj, -1.73, z)
    xyz = np.stack([x, y, z], 1) + rng.normal(0.0, 0.02, (n, 3))
    inten = rng.random(n)
    pts = np.concatenate([xyz, inten[:, None]], 1).astype(np.float32)
    return pts


def uniform_frame(seed: int, n: int = 24000, pc_range=KITTI_PC_RANGE) -> np.ndarray:
    """Cap-stress frame: n points uniform in range (exceeds 16000 distinct voxels)."""
    rng = np.random.default_rng(seed)
    lo = np.array(pc_range[:3], np.float64)
    hi = np.array(pc_range[3:], np.float64)
    xyz = lo + rng.random((n, 3)) * (hi - lo)
    inten = rng.random((n, 1))
    return np.concatenate([xyz, inten], 1).astype(np.float32)


def gt_boxes(seed: int, num_classes: int = 3, lo: int = 6, hi: int = 10):
    """GT boxes [M, 7] (x, y, z_bottom, dx, dy, dz, yaw) float32 and labels [M] int64."""
    rng = np.random.default_rng(10_000 + seed)
    m = int(rng.integers(lo, hi + 1))
    labels = rng.integers(0, num_classes, m)
    sizes = np.array(KITTI_SIZES, np.float64)[labels]
    x = rng.uniform(5.0, 65.0, m)
    y = rng.uniform(-35.0, 35.0, m)
    z = np.full(m, -1.73)
    yaw = rng.uniform(-np.pi, np.pi, m)
    boxes = np.concatenate([np.stack([x, y, z], 1), sizes, yaw[:, None]], 1)
    return boxes.astype(np.float32), labels.astype(np.int64)


def kitti_batch(batch: int, seed0: int = 0, num_classes: int = 3, cap_stress: bool = False):
    """B frames + GT; returns (list of [Ni,4] float32, list of boxes, list of labels)."""
    pts = [uniform_frame(seed0 + i) if cap_stress else kitti_frame(seed0 + i) for i in range(batch)]
    gts = [gt_boxes(seed0 + i, num_classes) for i in range(batch)]
    return pts, [g[0] for g in gts], [g[1] for g in gts]


# ---------------------------------------------------------------------- nuScenes (§8(f3), BASELINE config 4)
NUS_PC_RANGE = (-51.2, -51.2, -5.0, 51.2, 51.2, 3.0)
NUS_VOXEL_SIZE = (0.1, 0.1, 0.2)
NUS_CLASSES = ("car", "truck", "construction_vehicle", "bus", "trailer", "barrier", "motorcycle", "bicycle",
               "pedestrian", "traffic_cone")
# typical (x_size, y_size, z_size) per class
NUS_SIZES = ((4.6, 1.9, 1.7), (6.9, 2.5, 2.8), (6.4, 2.8, 3.2), (11.0, 2.9, 3.5), (12.3, 2.9, 3.9),
             (0.5, 2.5, 1.0), (2.1, 0.8, 1.5), (1.7, 0.6, 1.3), (0.7, 0.7, 1.8), (0.4, 0.4, 1.1))


def nus_frame(seed: int, sweeps: int = 10, keep: float = 0.7) -> np.ndarray:
    """HDL-32E-like multi-sweep frame, float32 [N, 5] (x, y, z, intensity, time lag): 32 beams at
    -30.67°..+10.67°, 360° azimuth in 0.33° steps, ground at z = -1.84 m, 15 % object returns at
    U(3, 50) m, background U(20, 80) m; sweep s is lagged by 0.05 s and shifted by 5 m/s ego motion."""
    rng = np.random.default_rng(50_000 + seed)
    elev = np.deg2rad(np.linspace(-30.67, 10.67, 32))
    azim = np.deg2rad(np.arange(-180.0, 180.0, 0.33))
    el, az = np.meshgrid(elev, azim, indexing="ij")
    el, az = el.ravel(), az.ravel()
    out = []
    for s in range(sweeps):
        m = rng.random(el.shape[0]) < keep
        e, a = el[m], az[m]
        n = e.shape[0]
        r = rng.uniform(20.0, 80.0, n)
        down = e < 0
        rg = np.where(down, 1.84 / np.tan(np.maximum(-e, 1e-6)), np.inf)
        ground = down & (rg < 80.0)
        r = np.where(ground, rg, r)
        obj = rng.random(n) < 0.15
        r = np.where(obj, np.minimum(rng.uniform(3.0, 50.0, n), r), r)
        x = r * np.cos(e) * np.cos(a) - 5.0 * 0.05 * s
        y = r * np.cos(e) * np.sin(a)
        z = np.where(ground & ~obj, -1.84, r * np.sin(e))
        xyz = np.stack([x, y, z], 1) + rng.normal(0.0, 0.02, (n, 3))
        inten = rng.uniform(0.0, 100.0, (n, 1))
        lag = np.full((n, 1), 0.05 * s)
        out.append(np.concatenate([xyz, inten, lag], 1))
    return np.concatenate(out, 0).astype(np.float32)


def nus_gt_boxes(seed: int, lo: int = 20, hi: int = 40):
    """GT boxes [M, 9] (x, y, z_bottom, dx, dy, dz, yaw, vx, vy) float32 and labels [M] int64."""
    rng = np.random.default_rng(60_000 + seed)
    m = int(rng.integers(lo, hi + 1))
    labels = rng.integers(0, len(NUS_CLASSES), m)
    sizes = np.array(NUS_SIZES, np.float64)[labels] * rng.uniform(0.9, 1.1, (m, 1))
    xy = rng.uniform(-50.0, 50.0, (m, 2))
    z = np.full((m, 1), -1.84)
    yaw = rng.uniform(-np.pi, np.pi, (m, 1))
    vel = rng.normal(0.0, 2.0, (m, 2))
    boxes = np.concatenate([xy, z, sizes, yaw, vel], 1)
    return boxes.astype(np.float32), labels.astype(np.int64)
