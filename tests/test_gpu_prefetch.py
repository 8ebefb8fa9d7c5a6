"""Trainer.train_step(next_points=...): the next batch's hard voxelisation queued on a side stream and
its voxel count read one step later must give the same training trajectory as voxelising inside
each step (same kernels, same inputs; only the stream they are queued on and the read point move).
Also: a prefetch for points that are not the next step's is dropped, and the step voxelises normally."""
import pytest
import torch

from robustpointclouds_amd.anchor_head import pack_gt
from robustpointclouds_amd.synthetic import kitti_batch
from robustpointclouds_amd.trainer import Trainer, make_kitti_model

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


def _batches(n, B=2):
    out = []
    for j in range(n):
        pts, boxes, labels = kitti_batch(B, seed0=100 + j * B, num_classes=1)
        gb, gl = pack_gt(list(zip(boxes, labels)), DEV)
        out.append(([torch.from_numpy(p).to(DEV) for p in pts], dict(gt_boxes=gb, gt_labels=gl)))
    return out


def _run(data, prefetch, order):
    torch.manual_seed(0)
    model = make_kitti_model(num_classes=1, device=DEV, epoch=3)
    tr = Trainer(model, bf16=True, device=DEV)
    logs = []
    for k, i in enumerate(order):
        nxt = data[order[k + 1]][0] if (prefetch and k + 1 < len(order)) else None
        logs.append({key: float(v) for key, v in tr.train_step(*data[i], next_points=nxt).items()})
    torch.cuda.synchronize()
    return logs, {k: v.detach().clone() for k, v in model.named_parameters()}


def _compare(a, b):
    la, pa = a
    lb, pb = b
    for x, y in zip(la, lb):
        assert set(x) == set(y)
        for k in x:
            assert abs(x[k] - y[k]) <= 1e-5 * max(1.0, abs(x[k])), (k, x[k], y[k])
    for k in pa:
        d = (pa[k] - pb[k]).abs().max().item()
        assert d <= 1e-6 * max(1.0, pa[k].abs().max().item()), (k, d)


def test_prefetch_same_trajectory():
    data = _batches(3)
    order = [0, 1, 2, 0]
    _compare(_run(data, False, order), _run(data, True, order))


def test_prefetch_for_other_points_is_dropped():
    data = _batches(2)
    torch.manual_seed(0)
    model = make_kitti_model(num_classes=1, device=DEV, epoch=3)
    tr = Trainer(model, bf16=True, device=DEV)
    tr.train_step(*data[0], next_points=data[1][0])
    assert tr._pending is not None and tr._pending[0] is data[1][0]
    log = tr.train_step(*data[0])          # not the prefetched points: voxelised in the step
    assert tr._pending is None
    assert all(torch.isfinite(torch.as_tensor(float(v))) for v in log.values())
