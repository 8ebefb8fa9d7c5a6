"""oracle/voxelize_ref.c (mmcv hard_voxelize restated in C) against an independent
pure-Python loop, on small frames that hit every branch: out-of-range points, the
max_voxels cap, the max_points cap, exact voxel boundaries, empty frames."""
import numpy as np
import pytest

from oracle import voxelize as ov
from robustpointclouds_amd.synthetic import KITTI_PC_RANGE, KITTI_VOXEL_SIZE, kitti_frame, uniform_frame


def _same(a, b):
    for x, y in zip(a, b):
        assert x.shape == y.shape and np.array_equal(x, y)


@pytest.mark.parametrize("seed", [0, 1])
def test_c_oracle_equals_python_loop_on_subsampled_frame(seed):
    pts = kitti_frame(seed)[::7][:3000]
    _same(ov.hard_voxelize(pts, KITTI_VOXEL_SIZE, KITTI_PC_RANGE, 5, 16000),
          ov.hard_voxelize_py(pts, KITTI_VOXEL_SIZE, KITTI_PC_RANGE, 5, 16000))


def test_caps_engage():
    rng = np.random.default_rng(3)
    # many points in few voxels (max_points cap) + more voxels than max_voxels
    base = np.array([[10.0, 0.0, -1.0, 0.5]], np.float32)
    dense = base + rng.uniform(0, 0.049, (200, 4)).astype(np.float32) * np.array([1, 1, 0, 1], np.float32)
    pts = np.concatenate([dense, uniform_frame(4, 2000)])
    a = ov.hard_voxelize(pts, KITTI_VOXEL_SIZE, KITTI_PC_RANGE, 5, 300)
    b = ov.hard_voxelize_py(pts, KITTI_VOXEL_SIZE, KITTI_PC_RANGE, 5, 300)
    _same(a, b)
    assert a[0].shape[0] == 300 and a[2].max() == 5


def test_boundaries_and_empty():
    vs, rg = KITTI_VOXEL_SIZE, KITTI_PC_RANGE
    pts = np.array([[0.0, -40.0, -3.0, 1.0],       # exactly at range min -> voxel 0
                    [70.4, 0.0, 0.0, 1.0],        # at range max -> rejected
                    [70.39999, 39.99999, 0.99999, 1.0],
                    [-1e-6, 0.0, 0.0, 1.0],       # just below min -> rejected
                    [np.nan, 0.0, 0.0, 1.0],
                    [5.0, 5.0, np.inf, 1.0]], np.float32)
    _same(ov.hard_voxelize(pts, vs, rg, 5, 100), ov.hard_voxelize_py(pts, vs, rg, 5, 100))
    v, c, n = ov.hard_voxelize(np.zeros((0, 4), np.float32), vs, rg, 5, 100)
    assert v.shape == (0, 5, 4) and c.shape == (0, 3) and n.shape == (0,)
