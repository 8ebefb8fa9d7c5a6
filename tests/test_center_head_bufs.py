"""CPU checks of CenterHead's persistent separate-head buffers (center_head._HeadBufs): the views a forward
hands the dense engine hold each task's BatchNorm parameters / running statistics and final-conv biases in
_BOX_ORDER, write_back returns the statistics to the modules, and a copied module builds its own buffers."""
import copy

import torch

from robustpointclouds_amd import center_head as ch


def _head():
    torch.manual_seed(0)
    h = ch.CenterHead(in_channels=64)
    for m in h.modules():
        if isinstance(m, torch.nn.BatchNorm2d):
            for t in (m.weight, m.bias):
                t.data.uniform_(-1, 1)
            m.running_mean.uniform_(-1, 1)
            m.running_var.uniform_(0.5, 2)
        if isinstance(m, torch.nn.Conv2d) and m.bias is not None:
            m.bias.data.uniform_(-1, 1)
    return h


def test_views_match_modules():
    h = _head()
    hb = ch._head_bufs(h, torch.device("cpu"))
    for t, th in enumerate(h.task_heads):
        cms = [getattr(th.task_head, n)[0] for n in ch._BOX_ORDER]
        fcs = [getattr(th.task_head, n)[1] for n in ch._BOX_ORDER]
        v = hb.views[t]
        assert torch.equal(v.weight, torch.cat([c.bn.weight.detach() for c in cms]))
        assert torch.equal(v.bias, torch.cat([c.bn.bias.detach() for c in cms]))
        assert torch.equal(v.running_mean, torch.cat([c.bn.running_mean for c in cms]))
        assert torch.equal(v.running_var, torch.cat([c.bn.running_var for c in cms]))
        assert torch.equal(hb.fviews[t], torch.cat([f.bias.detach() for f in fcs]))
    # the kernels update the running statistics in the buffers; write_back returns them
    hb.rm.add_(1.0)
    hb.rv.mul_(2.0)
    before = [(b.running_mean.clone(), b.running_var.clone()) for b in hb.bns]
    hb.write_back()
    for b, (m, v) in zip(hb.bns, before):
        assert torch.equal(b.running_mean, m + 1.0) and torch.equal(b.running_var, v * 2.0)
    # a second forward re-reads the modules (parameter updates between steps)
    th0 = h.task_heads[0]
    getattr(th0.task_head, ch._BOX_ORDER[0])[0].bn.weight.data.fill_(3.0)
    assert ch._head_bufs(h, torch.device("cpu")) is hb
    assert float(hb.views[0].weight[0]) == 3.0


def test_copy_builds_own_buffers():
    h = _head()
    hb = ch._head_bufs(h, torch.device("cpu"))
    h2 = copy.deepcopy(h)
    assert h2.__dict__.get("_head_bufs") is None
    hb2 = ch._head_bufs(h2, torch.device("cpu"))
    assert hb2 is not hb and hb2.w.data_ptr() != hb.w.data_ptr()
