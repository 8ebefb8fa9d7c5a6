"""HIP graphs over the dense part (dense_bev._graph_run): training steps that replay the captured
SECOND / SECONDFPN forward and SECOND backward graphs give bit-identical parameters and losses to the
same steps run eagerly (same kernels, same inputs, deterministic reductions), and the graphs are
actually captured and replayed."""
import copy

import pytest
import torch

from robustpointclouds_amd import dense_bev
from robustpointclouds_amd.anchor_head import pack_gt
from robustpointclouds_amd.synthetic import kitti_batch
from robustpointclouds_amd.trainer import Trainer, make_kitti_model

pytestmark = pytest.mark.gpu


def _data(dev, n):
    out = []
    for j in range(n):
        pts, boxes, labels = kitti_batch(6, seed0=100 + 6 * j, num_classes=3)
        gb, gl = pack_gt(list(zip(boxes, labels)), dev)
        out.append(([torch.from_numpy(p).to(dev) for p in pts], dict(gt_boxes=gb, gt_labels=gl)))
    return out


def test_graph_replay_bit_identical_to_eager():
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    m_graph = make_kitti_model(num_classes=3, device=dev, epoch=3)
    m_eager = copy.deepcopy(m_graph)
    t_graph = Trainer(m_graph, bf16=True, device=dev)
    t_eager = Trainer(m_eager, bf16=True, device=dev)
    data = _data(dev, 2)
    saved = dense_bev.GRAPHS
    logs = {}
    try:
        for name, tr, flag in (("graph", t_graph, True), ("eager", t_eager, False)):
            dense_bev.GRAPHS = flag
            logs[name] = [tr.train_step(*data[i % 2]) for i in range(5)]
            torch.cuda.synchronize()
    finally:
        dense_bev.GRAPHS = saved
    ents = [e for mod in (m_graph.backbone, m_graph.neck) for e in dense_bev.graph_cache(mod).values()
            if isinstance(e, dense_bev._GraphEntry)]
    assert len(ents) == 2 and all(e.graph is not None and e.calls == 5 for e in ents)
    assert any(b.graph is not None for e in ents for b in e.bwd.values())
    for a, b in zip(logs["graph"], logs["eager"]):
        for k in a:
            assert torch.equal(torch.as_tensor(a[k]), torch.as_tensor(b[k])), k
    for (n, p), (_, q) in zip(m_graph.named_parameters(), m_eager.named_parameters()):
        assert torch.equal(p, q), n
    for (n, p), (_, q) in zip(m_graph.named_buffers(), m_eager.named_buffers()):
        assert torch.equal(p, q), n


def test_rebuilt_model_never_replays_a_dropped_models_graph():
    """graphs live in each module's own cache, keyed by the addresses of its parameters
    and buffers — a model built after another one was dropped (its allocations may land on the
    freed addresses, its modules may reuse the ids) captures its own graphs: bit-identical to eager."""
    import gc
    dev = torch.device("cuda", 0)
    data = _data(dev, 2)
    saved = dense_bev.GRAPHS
    try:
        dense_bev.GRAPHS = True
        torch.manual_seed(1)
        m_old = make_kitti_model(num_classes=3, device=dev, epoch=3)
        t_old = Trainer(m_old, bf16=True, device=dev)
        for i in range(3):
            t_old.train_step(*data[i % 2])
        torch.cuda.synchronize()
        del t_old, m_old
        gc.collect()
        torch.manual_seed(2)
        m_new = make_kitti_model(num_classes=3, device=dev, epoch=3)
        m_ref = copy.deepcopy(m_new)
        t_new = Trainer(m_new, bf16=True, device=dev)
        t_ref = Trainer(m_ref, bf16=True, device=dev)
        logs_new = [t_new.train_step(*data[i % 2]) for i in range(3)]
        torch.cuda.synchronize()
        dense_bev.GRAPHS = False
        logs_ref = [t_ref.train_step(*data[i % 2]) for i in range(3)]
        torch.cuda.synchronize()
    finally:
        dense_bev.GRAPHS = saved
    for a, b in zip(logs_new, logs_ref):
        for k in a:
            assert torch.equal(torch.as_tensor(a[k]), torch.as_tensor(b[k])), k
    for (n, p), (_, q) in zip(m_new.named_parameters(), m_ref.named_parameters()):
        assert p.grad is None and torch.equal(p, q), n
    assert len([e for e in dense_bev.graph_cache(m_new.backbone).values() if isinstance(e, dense_bev._GraphEntry)]) == 1
