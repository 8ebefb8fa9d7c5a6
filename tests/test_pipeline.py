"""§8(f2) training pipeline on the GPU: LoadPointsFromFile (.bin), RandomFlip3D, GlobalRotScaleTrans,
PointsRangeFilter, ObjectRangeFilter, PointShuffle (configs/_base_/kitti-3d-car.py:42-68).

CPU: the `.bin` loader and the oracle restatement on hand-checked cases. GPU: rpc_augment_points /
rpc_augment_boxes against oracle/pipeline.py on synthetic KITTI frames — surviving points, their order
and the per-frame offsets exactly equal (the oracle writes the rotation with the kernel's op order),
boxes exactly, labels exactly; the device shuffle is a per-frame permutation of the same rows,
reproducible from its seed; rows past the survivors are NaN (dropped by hard_voxelize).
Upstream mmdet3d is not vendored: parity w.r.t. upstream itself is unpinned.
"""
import numpy as np
import pytest
import torch

from oracle.pipeline import augment_frame
from robustpointclouds_amd.pipeline import AUG_DTYPE, GpuTrainAugment, concat_frames, load_points_from_file
from robustpointclouds_amd.synthetic import KITTI_PC_RANGE, kitti_batch

R = [float(v) for v in KITTI_PC_RANGE]


def test_load_points_from_file(tmp_path):
    a = np.arange(40, dtype=np.float32).reshape(10, 4)
    f = tmp_path / "000001.bin"
    a.tofile(f)
    np.testing.assert_array_equal(load_points_from_file(str(f)), a)
    np.testing.assert_array_equal(load_points_from_file(str(f), load_dim=4, use_dim=3), a[:, :3])
    b = np.arange(50, dtype=np.float32).reshape(10, 5)   # NuScenes-style records, 4 columns kept
    b.tofile(f)
    np.testing.assert_array_equal(load_points_from_file(str(f), load_dim=5, use_dim=[0, 1, 2, 3]), b[:, :4])
    with pytest.raises(ValueError):
        load_points_from_file(str(f), load_dim=3)


def _frame(flip_h=0, flip_v=0, rot=0.0, scale=1.0, t=(0.0, 0.0, 0.0)):
    fr = np.zeros(1, AUG_DTYPE)[0]
    ang = torch.tensor(rot, dtype=torch.float32)
    fr["flip_h"], fr["flip_v"], fr["rot"] = flip_h, flip_v, rot
    fr["cosr"], fr["sinr"], fr["scale"] = float(torch.cos(ang)), float(torch.sin(ang)), scale
    fr["tx"], fr["ty"], fr["tz"] = t
    return fr


def test_oracle_known_transforms():
    pts = torch.tensor([[10.0, 5.0, -1.0, 0.3], [10.0, -5.0, 0.5, 0.1], [-1.0, 0.0, 0.0, 0.2]])
    boxes = torch.tensor([[10.0, 5.0, -1.0, 3.9, 1.6, 1.5, 0.2]])
    labels = torch.tensor([0])
    p, b, l = augment_frame(pts, boxes, labels, _frame(flip_h=1), R)
    assert torch.equal(p[:, 1], torch.tensor([-5.0, 5.0])) and p.shape[0] == 2      # x = -1 is filtered out
    assert float(b[0, 1]) == -5.0 and abs(float(b[0, 6]) + 0.2) < 1e-7
    p, b, l = augment_frame(pts[:2], boxes, labels, _frame(rot=float(np.pi / 2)), R)   # (10, 5) -> (-5, 10): out
    assert p.shape[0] == 1 and abs(float(p[0, 0]) - 5.0) < 1e-5 and abs(float(p[0, 1]) - 10.0) < 1e-5
    assert int(l[0]) == -1 and float(b[0, 3]) == 1.0                               # box centre left the range
    p, b, l = augment_frame(pts, boxes, labels, _frame(scale=2.0, t=(1.0, 0.0, 0.0)), R)
    assert torch.allclose(p[0, :3], torch.tensor([21.0, 10.0, -2.0])) and float(p[0, 3]) == np.float32(0.3)
    assert torch.allclose(b[0, :6], torch.tensor([21.0, 10.0, -2.0, 7.8, 3.2, 3.0]))
    p, b, l = augment_frame(pts, boxes, labels, _frame(rot=3.0), R)                 # yaw 3.2 -> 3.2 - 2 pi
    assert abs(float(b[0, 6]) - (0.2 + 3.0 - 2 * np.pi)) < 1e-5 or int(l[0]) == -1


def _batch(B, seed, dev):
    pts, boxes, labels = kitti_batch(B, seed0=seed, num_classes=3)
    M = max(len(b) for b in boxes)
    gb = torch.zeros(B, M, 7)
    gl = torch.full((B, M), -1, dtype=torch.long)
    gb[..., 3:6] = 1.0
    for i, (b, l) in enumerate(zip(boxes, labels)):
        gb[i, :len(b)] = torch.from_numpy(np.asarray(b, np.float32))
        gl[i, :len(l)] = torch.from_numpy(np.asarray(l, np.int64))
    return pts, gb, gl


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [0, 5])
def test_gpu_augment_matches_oracle(seed):
    dev = torch.device("cuda")
    B = 4
    pts, gb, gl = _batch(B, 40 + seed, dev)
    aug = GpuTrainAugment(R, shuffle=None, translation_std=(0.2, 0.2, 0.1), flip_ratio_bev_vertical=0.3)
    frames = aug.sample(B, np.random.RandomState(seed))
    x, off = concat_frames(pts, dev)
    gbd, gld = gb.clone().to(dev), gl.clone().to(dev)
    out, out_off, gbd, gld = aug(x, off, gbd, gld, frames=frames)
    out, out_off = out.cpu(), out_off.cpu().numpy()
    n = 0
    for b in range(B):
        rp, rb, rl = augment_frame(torch.from_numpy(pts[b]), gb[b], gl[b], frames[b], R)
        assert out_off[b] == n
        got = out[out_off[b]:out_off[b + 1]]
        assert got.shape == rp.shape
        assert torch.equal(got, rp), (b, (got - rp).abs().max())
        n += rp.shape[0]
        assert torch.equal(gld[b].cpu(), rl)
        assert torch.equal(gbd[b].cpu(), rb)
    assert out_off[B] == n
    assert torch.isnan(out[n:]).all()


@pytest.mark.gpu
def test_gpu_shuffle_is_a_seeded_permutation_per_frame():
    dev = torch.device("cuda")
    B = 3
    pts, gb, gl = _batch(B, 7, dev)
    x, off = concat_frames(pts, dev)
    fr = GpuTrainAugment(R, shuffle=None).sample(B, np.random.RandomState(1))
    plain, o1, _, _ = GpuTrainAugment(R, shuffle=None)(x, off, frames=fr)
    s1, o2, _, _ = GpuTrainAugment(R, shuffle="device")(x, off, frames=fr, seed=11)
    s1b, _, _, _ = GpuTrainAugment(R, shuffle="device")(x, off, frames=fr, seed=11)
    s2, _, _, _ = GpuTrainAugment(R, shuffle="device")(x, off, frames=fr, seed=12)
    assert torch.equal(o1, o2)
    o = o1.cpu().numpy()
    n = int(o[B])
    assert torch.isnan(s1[n:]).all()
    assert torch.equal(s1[:n], s1b[:n]) and not torch.equal(s1[:n], s2[:n])
    for b in range(B):
        a = plain[o[b]:o[b + 1]].cpu().numpy()
        c = s1[o[b]:o[b + 1]].cpu().numpy()
        assert not np.array_equal(a, c)
        np.testing.assert_array_equal(a[np.lexsort(a.T[::-1])], c[np.lexsort(c.T[::-1])])
