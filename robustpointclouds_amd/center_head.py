"""CenterHead training targets and losses on the HIP kernels.

Mirrors upstream mmdet3d `CenterHead.loss_by_feat` (targets from `get_targets_single`,
GaussianFocalLoss on clamp_sigmoid heatmaps, L1Loss on the boxes gathered at the GT centres) as
configured by the nuScenes base of configs/adversarial/adversarial-centerpoint_voxel-nuscenes.py:11-13
and called at models/detectors/adversarial_centerpoint.py:224. The whole loss (targets included) is
one autograd node over csrc/center_head.hip: heatmap logits [cells, hm_pitch] and boxes
[cells, box_pitch] in, the 2 * ntasks losses out; no host synchronisation (num_pos, the box count
and both normalisers stay on the device).
"""
from __future__ import annotations

import ctypes as C

import torch

from . import _ffi

NUS_TASKS = (("car",), ("truck", "construction_vehicle"), ("bus", "trailer"), ("barrier",),
             ("motorcycle", "bicycle"), ("pedestrian", "traffic_cone"))

# train_cfg.pts of centerpoint_voxel01_second_secfpn_head-dcn (nuScenes)
NUS_TRAIN_CFG = dict(grid_size=[1024, 1024, 40], voxel_size=[0.1, 0.1, 0.2], out_size_factor=8, dense_reg=1,
                     gaussian_overlap=0.1, max_objs=500, min_radius=2,
                     code_weights=[1.0, 1.0, 1.0, 1.0, 1.0, 1.0, 1.0, 1.0, 0.2, 0.2],
                     point_cloud_range=[-51.2, -51.2, -5.0, 51.2, 51.2, 3.0])


def center_cfg(tasks, train_cfg, B, H, W, hm_pitch, box_pitch, norm_bbox=True, loss_cls_weight=1.0,
               loss_bbox_weight=0.25) -> _ffi.RpcCenterCfg:
    if len(tasks) > 8:
        raise ValueError("at most 8 CenterHead tasks")
    c = _ffi.RpcCenterCfg()
    c.B, c.H, c.W = B, H, W
    c.ntasks = len(tasks)
    c.ncls_total = sum(len(t) for t in tasks)
    for i, t in enumerate(tasks):
        c.task_ncls[i] = len(t)
    c.max_objs = int(train_cfg["max_objs"]) * int(train_cfg.get("dense_reg", 1))
    c.min_radius = int(train_cfg["min_radius"])
    c.out_size_factor = int(train_cfg["out_size_factor"])
    c.norm_bbox = int(bool(norm_bbox))
    vs, pr = train_cfg["voxel_size"], train_cfg["point_cloud_range"]
    c.voxel_x, c.voxel_y, c.pc_x, c.pc_y = float(vs[0]), float(vs[1]), float(pr[0]), float(pr[1])
    c.gaussian_overlap = float(train_cfg["gaussian_overlap"])
    cw = train_cfg.get("code_weights") or [1.0] * 10
    for i in range(10):
        c.code_weights[i] = float(cw[i])
    c.loss_cls_weight, c.loss_bbox_weight = float(loss_cls_weight), float(loss_bbox_weight)
    c.hm_pitch, c.box_pitch = hm_pitch, box_pitch
    return c


def pack_gt(gt_boxes_list, gt_labels_list, device):
    """Per-frame [n, 9] LiDAR boxes / [n] labels -> padded device tensors [B, M, 9] fp32 and [B, M]
    int64 (-1 padding), built on the host in pinned memory and uploaded without a stream drain."""
    B = len(gt_boxes_list)
    M = max([int(b.shape[0]) for b in gt_boxes_list] + [1])
    boxes = torch.zeros((B, M, 9), dtype=torch.float32, pin_memory=torch.cuda.is_available())
    labels = torch.full((B, M), -1, dtype=torch.int64, pin_memory=torch.cuda.is_available())
    for i, (b, l) in enumerate(zip(gt_boxes_list, gt_labels_list)):
        n = int(b.shape[0])
        if n:
            boxes[i, :n] = b.detach().to("cpu", torch.float32)[:, :9]
            labels[i, :n] = l.detach().to("cpu", torch.int64)
    return boxes.to(device, non_blocking=True), labels.to(device, non_blocking=True)


class CenterLossFn(torch.autograd.Function):
    """(hm [cells, hm_pitch], box [cells, box_pitch]) -> losses [2 * ntasks] (heatmap, bbox per task)."""

    @staticmethod
    def forward(ctx, hm, box, gt_boxes, gt_labels, cfg):
        lib = _ffi.load()
        hm = hm.float().contiguous()
        box = box.float().contiguous()
        cells = cfg.B * cfg.H * cfg.W
        if hm.numel() != cells * cfg.hm_pitch or box.numel() != cells * cfg.box_pitch:
            raise ValueError("CenterLossFn: head output sizes do not match the config")
        maxg = int(gt_labels.shape[1])
        wsz = lib.rpc_center_head_workspace_size(C.byref(cfg), maxg)
        if wsz == 0:
            raise ValueError("CenterLossFn: invalid RpcCenterCfg")
        ws = _ffi.workspace(wsz, hm.device)
        out = torch.empty(2 * cfg.ntasks, dtype=torch.float32, device=hm.device)
        _ffi.check(lib.rpc_center_head_loss_forward(C.byref(cfg), _ffi.ptr(gt_boxes), _ffi.ptr(gt_labels), maxg,
                                                    _ffi.ptr(hm), _ffi.ptr(box), _ffi.ptr(out), _ffi.ptr(ws), wsz,
                                                    _ffi.stream_of(hm)), "rpc_center_head_loss_forward")
        ctx.save_for_backward(hm, box)
        ctx.ws, ctx.wsz, ctx.cfg = ws, wsz, cfg
        return out

    @staticmethod
    def backward(ctx, gl):
        lib = _ffi.load()
        hm, box = ctx.saved_tensors
        gl = gl.float().contiguous()
        dhm = torch.empty_like(hm)
        dbox = torch.empty_like(box)
        _ffi.check(lib.rpc_center_head_loss_backward(C.byref(ctx.cfg), _ffi.ptr(hm), _ffi.ptr(box), _ffi.ptr(gl),
                                                     _ffi.ptr(dhm), _ffi.ptr(dbox), _ffi.ptr(ctx.ws), ctx.wsz,
                                                     _ffi.stream_of(hm)), "rpc_center_head_loss_backward")
        ctx.ws = None
        return dhm, dbox, None, None, None


def center_targets(cfg, ws, maxg):
    """Views of the targets kept in a forward workspace: heatmap [B, H, W, ncls], ind / mask
    [B, T, max_objs], anno [B, T, max_objs, 10] (device tensors sharing the workspace)."""
    lib = _ffi.load()
    ptrs = [C.c_void_p() for _ in range(4)]
    _ffi.check(lib.rpc_center_head_targets(C.byref(cfg), maxg, _ffi.ptr(ws), *[C.byref(p) for p in ptrs]),
               "rpc_center_head_targets")
    base = ws.data_ptr()
    B, H, W, T, MO, N = cfg.B, cfg.H, cfg.W, cfg.ntasks, cfg.max_objs, cfg.ncls_total

    def view(p, dtype, shape):
        off = p.value - base
        n = 1
        for s in shape:
            n *= s
        esz = torch.tensor([], dtype=dtype).element_size()
        return ws[off:off + n * esz].view(dtype).view(*shape)

    return (view(ptrs[0], torch.float32, (B, H, W, N)), view(ptrs[1], torch.int32, (B, T, MO)),
            view(ptrs[2], torch.int32, (B, T, MO)), view(ptrs[3], torch.float32, (B, T, MO, 10)))


# ---------------------------------------------------------------------- CenterHead module (HIP)
import math  # noqa: E402

from torch import nn  # noqa: E402

from . import dense_bev as db  # noqa: E402

NUS_COMMON_HEADS = dict(reg=(2, 2), height=(1, 2), dim=(3, 2), rot=(2, 2), vel=(2, 2))
_BOX_ORDER = ("reg", "height", "dim", "rot", "vel")     # anno_box channel order (loss_by_feat concat)
_PAD = 64                                               # padded output width of the small convs


class ConvModule(nn.Module):
    """mmcv ConvModule(conv 3x3 no bias, BN2d (eps 1e-5, momentum 0.1), ReLU) — kaiming fan_out init."""

    def __init__(self, ci, co):
        super().__init__()
        self.conv = nn.Conv2d(ci, co, 3, padding=1, bias=False)
        self.bn = nn.BatchNorm2d(co)
        nn.init.kaiming_normal_(self.conv.weight, mode="fan_out", nonlinearity="relu")


class DeformConv2dPack(nn.Module):
    """mmcv DeformConv2dPack(64, 64, 3, padding=1, groups=4): weight [64, 16, 3, 3] (uniform
    1/sqrt(in*k*k)), conv_offset = Conv2d(64, 18, 3, padding 1, bias) zero-initialised."""

    def __init__(self, in_channels=64, out_channels=64, kernel_size=3, padding=1, groups=4):
        super().__init__()
        if (in_channels, out_channels, kernel_size, padding, groups) != (64, 64, 3, 1, 4):
            raise NotImplementedError("the HIP DCN is built for DCN(64 -> 64, k 3, pad 1, groups 4)")
        self.groups = groups
        self.weight = nn.Parameter(torch.empty(out_channels, in_channels // groups, kernel_size, kernel_size))
        stdv = 1.0 / math.sqrt(in_channels * kernel_size * kernel_size)
        nn.init.uniform_(self.weight, -stdv, stdv)
        self.conv_offset = nn.Conv2d(in_channels, 2 * kernel_size * kernel_size, kernel_size, padding=padding,
                                     bias=True)
        nn.init.zeros_(self.conv_offset.weight)
        nn.init.zeros_(self.conv_offset.bias)


def _final_conv(ci, n, bias_fill=None):
    c = nn.Conv2d(ci, n, 3, padding=1, bias=True)
    if bias_fill is None:
        nn.init.kaiming_normal_(c.weight, mode="fan_out", nonlinearity="relu")
        nn.init.zeros_(c.bias)
    else:
        nn.init.constant_(c.bias, bias_fill)
    return c


class SeparateHead(nn.Module):
    """mmdet3d SeparateHead (num_conv 2, final_kernel 3): per head ConvModule + Conv2d(64 -> n, bias)."""

    def __init__(self, in_channels, heads, head_conv=64):
        super().__init__()
        self.heads = dict(heads)
        for name, (n, num_conv) in self.heads.items():
            if num_conv != 2:
                raise NotImplementedError("SeparateHead with num_conv = 2 is built")
            self.add_module(name, nn.Sequential(ConvModule(in_channels, head_conv), _final_conv(head_conv, n)))


class DCNSeparateHead(nn.Module):
    """mmdet3d DCNSeparateHead: feature_adapt_cls / _reg (DCN), cls_head (ConvModule + Conv2d, bias
    init_bias), task_head (SeparateHead on the reg features)."""

    def __init__(self, in_channels, num_cls, heads, head_conv=64, init_bias=-2.19):
        super().__init__()
        heads = {k: v for k, v in dict(heads).items() if k != "heatmap"}
        self.feature_adapt_cls = DeformConv2dPack(in_channels, in_channels)
        self.feature_adapt_reg = DeformConv2dPack(in_channels, in_channels)
        self.cls_head = nn.Sequential(ConvModule(in_channels, head_conv), _final_conv(head_conv, num_cls, init_bias))
        self.task_head = SeparateHead(in_channels, heads, head_conv)
        self.num_cls = num_cls


def _imgs(B, H, W):
    return (B, H, W), (B, H, W), (B, H, W)


def _reg_blockdiag(head):
    """Every task's five separate-head final convs (64 -> n_i, i over _BOX_ORDER, each reading its own
    64-channel slice of the 320-channel reg image) as ONE 320 -> sum(n_i) conv per task: the weight is
    block-diagonal (output rows of head i read only input channels 64 i .. 64 i + 63), so it does the
    same MACs as the five convs in one launch and its data gradient lands in the 320-channel image
    directly. Built for all tasks at once (one cat + one scatter): [tasks * nr, 5 * 64, 3, 3] fp32, and
    the (row, block) index of every real weight row for splitting the gradient back."""
    ws, blk = [], []
    for th in head.task_heads:
        for i, name in enumerate(_BOX_ORDER):
            w = getattr(th.task_head, name)[1].weight
            ws.append(w.detach().float().reshape(w.shape[0], -1))
            blk.extend([i] * w.shape[0])
    nb = len(_BOX_ORDER)
    Wall = torch.cat(ws)
    rows = Wall.shape[0]
    key = (rows, tuple(blk), Wall.device)
    idx = _BD_IDX.get(key)
    if idx is None:
        idx = (torch.arange(rows, device=Wall.device), torch.tensor(blk, device=Wall.device))
        _BD_IDX.clear()
        _BD_IDX[key] = idx
    Wbd = torch.zeros((rows, nb, Wall.shape[1]), dtype=torch.float32, device=Wall.device)
    Wbd[idx] = Wall
    return Wbd.view(rows, nb * 64, 3, 3), idx


_BD_IDX = {}


def _prep_head(eng, head, dev, st):
    """Every dense-engine weight operand of the head in batched launches (one launch per conv cost ~15 us
    each: 1.35 ms per CenterPoint step): key -> (forward, data-gradient) operands. Small convs are padded
    to 64 output channels in the kernel (RpcDenseWprep.co_src) instead of through a zero-filled fp32 copy.
    The 2 * tasks DCN offset convs (all reading the shared-conv image) are ONE 64 -> 18 * 2 * tasks conv
    ("offcat", padded to a multiple of 64 outputs), each task's five reg final convs one block-diagonal
    320 -> sum(n_i) conv ("regbd")."""
    items = []
    out = {}

    def add(conv, pad=False):
        W = conv.weight.detach().float().contiguous()
        co, ci = W.shape[0], W.shape[1]
        items.append((id(conv), W, ci, _PAD if pad else co, co if pad else 0))

    add(head.shared_conv.conv)
    offs = [dcn.conv_offset.weight.detach().float() for th in head.task_heads
            for dcn in (th.feature_adapt_cls, th.feature_adapt_reg)]
    Woff = torch.cat(offs).contiguous()
    nof = Woff.shape[0]
    items.append((("offcat",), Woff, Woff.shape[1], -(-nof // 64) * 64, nof))
    out[("offcat", "n")] = nof
    Wbd, bd_idx = _reg_blockdiag(head)
    out[("regbd", "idx")] = bd_idx
    nr = Wbd.shape[0] // len(head.task_heads)
    for t, th in enumerate(head.task_heads):
        add(th.cls_head[0].conv)
        add(th.cls_head[1], True)
        cms = [getattr(th.task_head, name)[0] for name in _BOX_ORDER]
        Wcat = torch.cat([cm.conv.weight.detach().float() for cm in cms]).contiguous()
        items.append((("regcat", id(th)), Wcat, Wcat.shape[1], Wcat.shape[0], 0))
        out[("regcat", id(th), "W")] = Wcat
        if nr > _PAD:
            raise NotImplementedError("CenterHead: more than 64 box channels per task")
        items.append((("regbd", id(th)), Wbd[nr * t:nr * (t + 1)], Wbd.shape[1], _PAD, nr))
    for g0 in range(0, len(items), 16):
        grp = items[g0:g0 + 16]
        descs = (_ffi.RpcDenseWprep * len(grp))()
        for i, (key, W, ci, co, co_src) in enumerate(grp):
            wf = torch.empty((9, co, ci), dtype=eng.dt, device=dev)
            wd = torch.empty((9, ci, co), dtype=eng.dt, device=dev)
            descs[i] = _ffi.RpcDenseWprep(W.data_ptr(), wf.data_ptr(), wd.data_ptr(), 0, ci, co, 9, 1, co_src)
            out[key] = (wf, wd)
        _ffi.check(eng.wprep_batch(descs, len(grp), st), "rpc_dense_wprep_batch")
    return out


class _CatBN:
    """The BatchNorm2d modules of k ConvModules that share their input, side by side as one 64k-channel
    BatchNorm for one wide conv + BN + ReLU launch sequence (the attributes dense_bev._forward_layer /
    _backward_layer read): views of a task's channels in the _HeadBufs buffers (the running statistics the
    kernels update go back to the modules through _HeadBufs.write_back)."""

    def __init__(self, bns, bufs, sl):
        self.bns = bns
        self.eps, self.momentum = float(bns[0].eps), float(bns[0].momentum)
        if any(float(b.eps) != self.eps or float(b.momentum) != self.momentum for b in bns):
            raise NotImplementedError("CenterHead: the separate-head BatchNorms must share eps / momentum")
        self.weight, self.bias = bufs.w[sl], bufs.b[sl]
        self.running_mean, self.running_var = bufs.rm[sl], bufs.rv[sl]


class _HeadBufs:
    """Every task's separate-head BatchNorms (tasks x 5 ConvModules of 64 channels: weight, bias, running mean / var)
    and final-conv biases in persistent flat buffers, filled by ONE multi-tensor copy per forward (was 5 cats per
    task: 30 launches per CenterPoint step), with per-task _CatBN-like views; write_back() returns every task's
    running statistics in one multi-tensor copy. Rebuilt when the modules or the device change."""

    @staticmethod
    def key_of(head, dev):
        return (str(dev),) + tuple(id(getattr(th.task_head, name)) for th in head.task_heads for name in _BOX_ORDER)

    def __init__(self, head, dev):
        self.key = self.key_of(head, dev)
        self.cms = [[getattr(th.task_head, name)[0] for name in _BOX_ORDER] for th in head.task_heads]
        self.fcs = [[getattr(th.task_head, name)[1] for name in _BOX_ORDER] for th in head.task_heads]
        self.bns = [cm.bn for cms in self.cms for cm in cms]
        self.fbs = [f.bias for fcs in self.fcs for f in fcs]
        nc = sum(b.num_features for b in self.bns)
        self.w, self.b, self.rm, self.rv = (torch.empty(nc, dtype=torch.float32, device=dev) for _ in range(4))
        self.fb = torch.empty(sum(f.numel() for f in self.fbs), dtype=torch.float32, device=dev)
        sz = [b.num_features for b in self.bns]
        fsz = [f.numel() for f in self.fbs]
        self.dst = (list(self.w.split(sz)) + list(self.b.split(sz)) + list(self.rm.split(sz)) + list(self.rv.split(sz))
                    + list(self.fb.split(fsz)))
        self.views, self.fviews = [], []
        c = f = 0
        for t, cms in enumerate(self.cms):
            n = sum(cm.bn.num_features for cm in cms)
            nf = sum(x.bias.numel() for x in self.fcs[t])
            self.views.append(_CatBN([cm.bn for cm in cms], self, slice(c, c + n)))
            self.fviews.append(self.fb[f:f + nf])
            c, f = c + n, f + nf

    # not part of a copied or pickled module (the copy builds its own on its first forward)
    def __deepcopy__(self, memo):
        return None

    def __reduce__(self):
        return (_no_bufs, ())

    def fill(self):
        src = ([b.weight.detach() for b in self.bns] + [b.bias.detach() for b in self.bns] +
               [b.running_mean for b in self.bns] + [b.running_var for b in self.bns] + [x.detach() for x in self.fbs])
        torch._foreach_copy_(self.dst, src)

    def write_back(self):
        sz = [b.num_features for b in self.bns]
        torch._foreach_copy_([b.running_mean for b in self.bns] + [b.running_var for b in self.bns],
                             list(self.rm.split(sz)) + list(self.rv.split(sz)))


def _no_bufs():
    return None


def _head_bufs(head, dev):
    hb = head.__dict__.get("_head_bufs")
    if hb is None or hb.key != _HeadBufs.key_of(head, dev):
        hb = head.__dict__["_head_bufs"] = _HeadBufs(head, dev)
    hb.fill()
    return hb


class _CatConv:
    def __init__(self, weight):
        self.weight = weight


def _conv_nobn_fwd(eng, weight, ci, h, pitch, B, H, W, dev, st, wts=None, n=None, co=_PAD):
    """3x3 conv (no BN) on the dense engine (bf16 or fp32) with the n real outputs padded to co ->
    (z image, record). wts: (forward, data-gradient) operands from _prep_head, else prepared here."""
    n = weight.shape[0] if n is None else n
    if wts is None:
        W32 = weight.detach().float().contiguous()
        wf = torch.empty((9, co, ci), dtype=eng.dt, device=dev)
        wd = torch.empty((9, ci, co), dtype=eng.dt, device=dev)
        desc = (_ffi.RpcDenseWprep * 1)(_ffi.RpcDenseWprep(W32.data_ptr(), wf.data_ptr(), wd.data_ptr(), 0, ci, co,
                                                           9, 1, n))
        _ffi.check(eng.wprep_batch(desc, 1, st), "rpc_dense_wprep_batch")
    else:
        wf, wd = wts
    z = db._image(B, co, H, W, dev, eng.dt)
    R = _ffi.int_arr((B, H, W))
    _ffi.check(eng.conv(db.S1, _ffi.ptr(h), pitch, ci, _ffi.ptr(wf), co, _ffi.ptr(z), co, 0, 0, None, R, R, R,
                        st), "rpc_dense_conv")
    return z, dict(h=h, pitch=pitch, wd=wd, ci=ci, n=n, co=co, B=B, H=H, W=W)


def _conv_nobn_bwd(eng, rec, dz, dev, st, need_dx=True, dx_out=None, accumulate=False, dx_pitch=None):
    """dz: the padded output gradient image (rec["co"] channels, the padding zero) -> (dx, dW[:n])."""
    ci, co, B, H, W = rec["ci"], rec["co"], rec["B"], rec["H"], rec["W"]
    R = _ffi.int_arr((B, H, W))
    dW = torch.empty((co, ci, 3, 3), dtype=torch.float32, device=dev)
    wsz = eng.wgrad_ws(db.S1, R, ci, co)
    ws = _ffi.workspace(wsz, dev)
    _ffi.check(eng.wgrad(db.S1, 0, _ffi.ptr(rec["h"]), rec["pitch"], ci, _ffi.ptr(dz), co, co, R, R, R,
                         _ffi.ptr(dW), _ffi.ptr(ws), wsz, st), "rpc_dense_wgrad")
    dx = None
    if need_dx:
        dx = dx_out if dx_out is not None else db._image(B, ci, H, W, dev, eng.dt)
        _ffi.check(eng.conv(db.S1, _ffi.ptr(dz), co, co, _ffi.ptr(rec["wd"]), ci, _ffi.ptr(dx), dx_pitch or ci, 0,
                            1 if accumulate else 0, None, R, R, R, st), "rpc_dense_conv(dgrad)")
    return dx, dW[:rec["n"]]


# test hook (tests/test_gpu_dcn_head.py): when a list, each training forward appends one entry per ConvModule
# BatchNorm — (module name, z [cells][co] pre-BN image, bn [4co] scale / beta / mean / invstd, channel slice, B,
# H, W) — from which the engine's exact ReLU decisions are recomputed (tests/_dense_masks.py engine_masks form)
DEBUG = None


def _debug(name, rec, sl, B, H, W):
    if DEBUG is not None:
        DEBUG.append((name, rec["z"].detach(), rec["bn"].detach(), sl, B, H, W))


def _conv_module_layer(cm):
    return db._Layer(db.S1, cm.conv, cm.bn, 0, cm.conv.in_channels, cm.conv.out_channels, 9)


class CenterHeadFn(torch.autograd.Function):
    """The whole CenterHead (shared conv + every DCNSeparateHead) as one node: neck image ->
    (hm [cells, hm_pitch], box [cells, box_pitch]) fp32; the shared feature gradient is accumulated in
    fp32 (DCN input gradients) plus the engine's dtype (offset-conv data gradients). The engine follows
    the neck image: bf16 (perf mode: bf16 dense engine + bf16-MFMA DCN) or fp32 (parity mode: fp32
    dense engine, fp32 DCN, fp32 head images)."""

    @staticmethod
    def forward(ctx, x, head, *params):
        lib = _ffi.load()
        dev = x.device
        st = _ffi.stream_of(x)
        eng = db._engine(lib, x)
        f32 = eng.f32
        xi = db._nhwc(x, eng.dt)
        B, Cin, H, W = xi.shape
        if H % 8 or W % 8:
            raise RuntimeError("HIP CenterHead needs a feature map with H, W multiples of 8")
        training = head.training
        cells = B * H * W
        hm = torch.empty((cells, head.hm_pitch), dtype=torch.float32, device=dev)
        box = torch.empty((cells, head.box_pitch), dtype=torch.float32, device=dev)
        pack = lib.rpc_head_pack_f32 if f32 else lib.rpc_head_pack
        prep = _prep_head(eng, head, dev, st)
        Lsh = _conv_module_layer(head.shared_conv)
        y0, rsh, _, _ = db._forward_layer(eng, Lsh, xi, Cin, B, H, W, training, dev, st,
                                          wts=prep[id(head.shared_conv.conv)])
        bns = [head.shared_conv.bn]
        if training:
            _debug("shared_conv", rsh, None, B, H, W)
        trecs = []
        c0 = 0
        # the DCN offsets of every task and branch: one 64 -> 18 * 2 * tasks conv of the shared image
        nof = prep[("offcat", "n")]
        cof = -(-nof // 64) * 64
        ozc, orec = _conv_nobn_fwd(eng, None, 64, y0, 64, B, H, W, dev, st, prep[("offcat",)], n=nof, co=cof)
        hbufs = _head_bufs(head, dev)
        for t, th in enumerate(head.task_heads):
            tr = {}
            for br, dcn in (("cls", th.feature_adapt_cls), ("reg", th.feature_adapt_reg)):
                j = 2 * t + (br == "reg")
                oz = ozc[:, 18 * j:18 * (j + 1)]
                ob = dcn.conv_offset.bias.detach().float().contiguous()
                feat = db._image(B, 64, H, W, dev, eng.dt)
                if f32:
                    wdd = dcn.weight.detach().float().contiguous()
                    _ffi.check(lib.rpc_dcn_forward_f32(_ffi.ptr(y0), 64, _ffi.ptr(oz), cof, _ffi.ptr(ob),
                                                       _ffi.ptr(wdd), _ffi.ptr(feat), 64, B, H, W, st),
                               "rpc_dcn_forward_f32")
                else:
                    wf = torch.empty((9, 64, 64), dtype=torch.bfloat16, device=dev)
                    wdd = torch.empty((9, 64, 64), dtype=torch.bfloat16, device=dev)
                    _ffi.check(lib.rpc_dcn_prep_weight(_ffi.ptr(dcn.weight.detach().float().contiguous()),
                                                       _ffi.ptr(wf), _ffi.ptr(wdd), st), "rpc_dcn_prep_weight")
                    _ffi.check(lib.rpc_dcn_forward(_ffi.ptr(y0), 64, _ffi.ptr(oz), cof, _ffi.ptr(ob), _ffi.ptr(wf),
                                                   _ffi.ptr(feat), 64, B, H, W, st), "rpc_dcn_forward")
                tr[br] = dict(dcn=dcn, oz=oz, j=j, wd=wdd, ob=ob, feat=feat)
            # cls branch -> heatmap logits
            L = _conv_module_layer(th.cls_head[0])
            hcls, rc, _, _ = db._forward_layer(eng, L, tr["cls"]["feat"], 64, B, H, W, training, dev, st,
                                               wts=prep[id(th.cls_head[0].conv)])
            bns.append(th.cls_head[0].bn)
            if training:
                _debug(f"task_heads.{t}.cls_head.0", rc, None, B, H, W)
            fc = th.cls_head[1]
            z, frec = _conv_nobn_fwd(eng, fc.weight, 64, hcls, 64, B, H, W, dev, st, prep[id(fc)])
            _ffi.check(pack(_ffi.ptr(z), _PAD, th.num_cls, _ffi.ptr(fc.bias.detach().float().contiguous()),
                                         _ffi.ptr(hm), head.hm_pitch, c0, cells, st), "rpc_head_pack")
            tr["cls_layers"] = (rc, frec, fc, c0, th.num_cls, hm, head.hm_pitch)
            c0 += th.num_cls
            # reg branches -> anno_box channels: the five ConvModules of the separate head share their input
            # (the DCN feature): one 64 -> 320 conv + BatchNorm + ReLU; the five final convs as one
            # block-diagonal 320 -> sum(n_i) conv whose outputs are the task's contiguous anno_box channels
            cms = hbufs.cms[t]
            cbn = hbufs.views[t]
            Lr = db._Layer(db.S1, _CatConv(prep[("regcat", id(th), "W")]), cbn, 0, 64, 64 * len(cms), 9)
            hr, rr, _, _ = db._forward_layer(eng, Lr, tr["reg"]["feat"], 64, B, H, W, training, dev, st,
                                             wts=prep[("regcat", id(th))])
            if training:
                for k, name in enumerate(_BOX_ORDER):
                    _debug(f"task_heads.{t}.task_head.{name}.0", rr, slice(64 * k, 64 * (k + 1)), B, H, W)
            bns.extend(cbn.bns)
            fcs = [getattr(th.task_head, name)[1] for name in _BOX_ORDER]
            nb = sum(f.weight.shape[0] for f in fcs)
            z, frec = _conv_nobn_fwd(eng, None, 64 * len(cms), hr, 64 * len(cms), B, H, W, dev, st,
                                     prep[("regbd", id(th))], n=nb)
            _ffi.check(pack(_ffi.ptr(z), _PAD, nb, _ffi.ptr(hbufs.fviews[t]), _ffi.ptr(box), head.box_pitch, 10 * t,
                            cells, st), "rpc_head_pack")
            tr["reg_cm"] = (rr, cms)
            tr["regs"] = (frec, fcs, 10 * t, nb)
            trecs.append(tr)
        if training:
            hbufs.write_back()
            _ffi.bump_batches(bns)
        ctx.head, ctx.rsh, ctx.trecs, ctx.orec = head, rsh, trecs, orec
        ctx.bd_idx = prep[("regbd", "idx")]
        ctx.shape = (B, H, W, Cin)
        ctx.f32 = f32
        ctx.param_list = params
        ctx.need_x = ctx.needs_input_grad[0]
        return hm, box

    @staticmethod
    def backward(ctx, ghm, gbox):
        lib = _ffi.load()
        B, H, W, Cin = ctx.shape
        g_any = ghm if ghm is not None else gbox
        dev = g_any.device
        st = _ffi.stream_of(g_any)
        cells = B * H * W
        head = ctx.head
        eng = db._Eng(lib, ctx.f32)
        f32 = eng.f32
        ghm = ghm.contiguous() if ghm is not None else torch.zeros((cells, head.hm_pitch), device=dev)
        gbox = gbox.contiguous() if gbox is not None else torch.zeros((cells, head.box_pitch), device=dev)
        grads = {}
        uwsz = lib.rpc_head_unpack_workspace_size()
        uws = _ffi.workspace(uwsz, dev)
        dY0f = torch.zeros((cells, 64), dtype=torch.float32, device=dev)     # DCN input gradients
        dwsz = lib.rpc_dcn_backward_workspace_size(B, H, W)
        dws = _ffi.workspace(dwsz, dev)
        orec = ctx.orec
        cof = orec["co"]
        # the concatenated offset conv's output gradient: every DCN writes its 18 channels (channel 18 j),
        # the padding channels stay zero
        doffc = torch.zeros((B, H, W, cof), dtype=eng.dt, device=dev).permute(0, 3, 1, 2)

        unpack = lib.rpc_head_unpack_grad_f32 if f32 else lib.rpc_head_unpack_grad

        def final_conv_bwd(frec, g, gp, off, n, dx_out=None, dx_pitch=None):
            dz = db._image(B, _PAD, H, W, dev, eng.dt)
            db_ = torch.empty(n, dtype=torch.float32, device=dev)
            _ffi.check(unpack(_ffi.ptr(g), gp, off, n, _ffi.ptr(dz), _PAD, cells, _ffi.ptr(db_),
                              _ffi.ptr(uws), uwsz, st), "rpc_head_unpack_grad")
            dh, dW = _conv_nobn_bwd(eng, frec, dz, dev, st, True, dx_out, False, dx_pitch)
            return dh, dW, db_

        rows, blk = ctx.bd_idx
        rb = 0
        for t, tr in enumerate(ctx.trecs):
            rc, frec, fc, c0, ncls, _, hp = tr["cls_layers"]
            dh, grads[id(fc.weight)], grads[id(fc.bias)] = final_conv_bwd(frec, ghm, hp, c0, ncls)
            dfc, dWc, dg, dbt, _ = db._backward_layer(eng, rc, dh, 64, 0, dev, st, True)
            L = rc["L"]
            grads[id(L.conv.weight)], grads[id(L.bnm.weight)], grads[id(L.bnm.bias)] = dWc, dg, dbt
            # reg: the block-diagonal final conv's data gradient is the 320-channel image of the concatenated
            # ConvModule; its weight gradient's diagonal blocks are the five final convs' (gathered in one op)
            rr, cms = tr["reg_cm"]
            nct = 64 * len(cms)
            frec2, fcs, bo, nb = tr["regs"]
            dh_cat, dWbd, dbb = final_conv_bwd(frec2, gbox, head.box_pitch, bo, nb)
            dWr = dWbd.reshape(nb, len(cms), -1)[rows[:nb], blk[rb:rb + nb]]
            rb += nb
            for f, w_, b_ in zip(fcs, dWr.split([f.weight.shape[0] for f in fcs]),
                                 dbb.split([f.weight.shape[0] for f in fcs])):
                grads[id(f.weight)], grads[id(f.bias)] = w_.view_as(f.weight), b_
            dfr, dWc, dg, dbt, _ = db._backward_layer(eng, rr, dh_cat, nct, 0, dev, st, True)
            for cm, w_, g_, b_ in zip(cms, dWc.split(64), dg.split(64), dbt.split(64)):
                grads[id(cm.conv.weight)], grads[id(cm.bn.weight)], grads[id(cm.bn.bias)] = w_, g_, b_
            for br, dfeat in (("cls", dfc), ("reg", dfr)):
                d = tr[br]
                dob = torch.empty(18, dtype=torch.float32, device=dev)
                dWd = torch.empty((64, 16, 3, 3), dtype=torch.float32, device=dev)
                dcn_bwd = lib.rpc_dcn_backward_f32_ex if f32 else lib.rpc_dcn_backward_ex
                _ffi.check(dcn_bwd(_ffi.ptr(orec["h"]), 64, _ffi.ptr(d["oz"]), cof, _ffi.ptr(d["ob"]), _ffi.ptr(d["wd"]),
                                   _ffi.ptr(dfeat), 64, _ffi.ptr(dY0f), _ffi.ptr(doffc[:, 18 * d["j"]:]), cof, 18,
                                   _ffi.ptr(dob), _ffi.ptr(dWd), B, H, W, _ffi.ptr(dws), dwsz, st), "rpc_dcn_backward")
                dcn = d["dcn"]
                grads[id(dcn.weight)] = dWd
                grads[id(dcn.conv_offset.bias)] = dob
        dY0b, dWo = _conv_nobn_bwd(eng, orec, doffc, dev, st, True)
        for t, tr in enumerate(ctx.trecs):
            for br in ("cls", "reg"):
                d = tr[br]
                grads[id(d["dcn"].conv_offset.weight)] = dWo[18 * d["j"]:18 * (d["j"] + 1)]
        dY0 = (dY0f + dY0b.permute(0, 2, 3, 1).reshape(cells, 64).float()).to(eng.dt)
        dY0 = dY0.view(B, H, W, 64).permute(0, 3, 1, 2)
        dx, dWs, dgs, dbs, _ = db._backward_layer(eng, ctx.rsh, dY0, 64, 0, dev, st, ctx.need_x)
        L = ctx.rsh["L"]
        grads[id(L.conv.weight)], grads[id(L.bnm.weight)], grads[id(L.bnm.bias)] = dWs, dgs, dbs
        ctx.trecs = ctx.rsh = ctx.orec = None
        return (dx, None) + tuple(grads.get(id(p)) for p in ctx.param_list)


class CenterHead(nn.Module):
    """upstream mmdet3d CenterHead with DCNSeparateHead task heads (nuScenes base of
    adversarial-centerpoint_voxel-nuscenes.py:11-13), on the HIP kernels only (no torch path):
    forward -> per-task prediction dicts (NCHW views of the packed fp32 head buffers);
    loss_by_feat -> CenterLossFn (csrc/center_head.hip). Parameter names follow mmdet3d."""

    def __init__(self, in_channels=512, tasks=None, common_heads=None, share_conv_channel=64, train_cfg=None,
                 test_cfg=None, norm_bbox=True, loss_cls_weight=1.0, loss_bbox_weight=0.25, init_bias=-2.19,
                 **kwargs):
        super().__init__()
        tasks = tasks or [dict(num_class=len(t), class_names=list(t)) for t in NUS_TASKS]
        self.class_names = [tuple(t["class_names"]) for t in tasks]
        self.num_classes = [len(c) for c in self.class_names]
        common_heads = dict(common_heads or NUS_COMMON_HEADS)
        if tuple(common_heads) != _BOX_ORDER:
            raise NotImplementedError("common_heads must be reg, height, dim, rot, vel (nuScenes)")
        self.shared_conv = ConvModule(in_channels, share_conv_channel)
        self.task_heads = nn.ModuleList([DCNSeparateHead(share_conv_channel, n, common_heads, 64, init_bias)
                                         for n in self.num_classes])
        self.train_cfg = dict(NUS_TRAIN_CFG, **(train_cfg or {}))
        self.test_cfg = test_cfg
        self.norm_bbox = norm_bbox
        self.loss_cls_weight, self.loss_bbox_weight = loss_cls_weight, loss_bbox_weight
        self.hm_pitch = sum(self.num_classes)
        self.box_pitch = 10 * len(self.num_classes)

    def hip_params(self):
        return [p for p in self.parameters()]

    def forward(self, feats):
        x = feats[0] if isinstance(feats, (list, tuple)) else feats
        if not x.is_cuda:
            raise RuntimeError("CenterHead runs on the HIP kernels only (no CPU path)")
        hm, box = CenterHeadFn.apply(x, self, *self.hip_params())
        B, _, H, W = x.shape
        hm4, box4 = hm.view(B, H, W, -1), box.view(B, H, W, -1)
        preds, c0 = [], 0
        for t, n in enumerate(self.num_classes):
            d, bo = {}, 10 * t
            for name, w in zip(_BOX_ORDER, (2, 1, 3, 2, 2)):
                d[name] = box4[..., bo:bo + w].permute(0, 3, 1, 2)
                bo += w
            d["heatmap"] = hm4[..., c0:c0 + n].permute(0, 3, 1, 2)
            d["_packed"] = (hm, box, B, H, W)
            c0 += n
            preds.append([d])
        return tuple(preds)

    def loss_by_feat(self, preds_dicts, batch_gt_instances_3d, *args, **kwargs):
        """batch_gt_instances_3d: per-frame instances (bboxes_3d [n, 9] LiDAR boxes, labels_3d) or the
        trainer's padded device dict(gt_boxes [B, M, 9], gt_labels [B, M], -1 padding)."""
        hm, box, B, H, W = preds_dicts[0][0]["_packed"]
        if isinstance(batch_gt_instances_3d, dict) and "gt_boxes" in batch_gt_instances_3d:
            gb = batch_gt_instances_3d["gt_boxes"].float().contiguous()
            gl = batch_gt_instances_3d["gt_labels"].long().contiguous()
        else:
            boxes = [g.bboxes_3d if hasattr(g, "bboxes_3d") else g["bboxes_3d"] for g in batch_gt_instances_3d]
            labels = [g.labels_3d if hasattr(g, "labels_3d") else g["labels_3d"] for g in batch_gt_instances_3d]
            boxes = [getattr(b, "tensor", b) for b in boxes]
            gb, gl = pack_gt(boxes, labels, hm.device)
        cfg = center_cfg([tuple(c) for c in self.class_names], self.train_cfg, B, H, W, self.hm_pitch, self.box_pitch,
                         self.norm_bbox, self.loss_cls_weight, self.loss_bbox_weight)
        lv = CenterLossFn.apply(hm, box, gb, gl, cfg)
        out = {}
        for t in range(len(self.num_classes)):
            out[f"task{t}.loss_heatmap"] = lv[2 * t]
            out[f"task{t}.loss_bbox"] = lv[2 * t + 1]
        out = PackedCenterLosses(out)
        out.packed = lv
        return out

    def loss(self, feats, batch_data_samples, **kwargs):
        preds = self(feats)
        if isinstance(batch_data_samples, dict):
            return self.loss_by_feat(preds, batch_data_samples)
        return self.loss_by_feat(preds, [s.gt_instances_3d if hasattr(s, "gt_instances_3d") else s["gt_instances_3d"]
                                         for s in batch_data_samples])


class PackedCenterLosses(dict):
    """task{t}.loss_heatmap / loss_bbox dict that also carries the device vector they are views of."""
    packed = None
