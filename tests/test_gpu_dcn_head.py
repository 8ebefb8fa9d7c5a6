"""§8(f3): the DCNSeparateHead deformable convolution (csrc/dcn.hip) and the whole HIP CenterHead
(shared conv + six DCN task heads on the dense engine) vs float64 CPU references.

DCN: oracle/dcn.py (mmcv deform_conv2d restated, autograd gradients) on the same bf16-rounded
input, offsets and weights; the kernel samples in fp32 and multiplies bf16 columns (fp32 accumulate),
so agreement is bf16-level: forward relative L2 <= 1e-2, gradients (input, offsets, offset bias,
weights) relative L2 <= 2e-2. Head: the same layer stack in float64 torch (conv / BatchNorm (batch
statistics) / ReLU / oracle DCN), outputs relative L2 <= 3e-2 and gradient directions (cosine)
>= 0.98 — the head runs in bf16 activations. Parity mode (fp32 neck image -> fp32 dense engine, fp32
DCN rpc_dcn_*_f32, fp32 head images): DCN forward relative L2 <= 1e-5 and gradients <= 1e-4 against the
float64 oracle on the same fp32 values; the whole head's outputs <= 1e-4, input gradient <= 1e-3 and every
parameter gradient <= 5e-3 (BatchNorm-backward cancellation), the float64 head evaluated on the engine's ReLU
decisions (same-branch parity, as tests/test_gpu_e2e_parity.py) with every decision it would take differently
within FLIP_PRE_MAX of zero. Parity w.r.t. mmcv / mmdet3d is unpinned
(not vendored)."""
import pytest
import torch
import torch.nn.functional as Fn

from oracle.dcn import deform_conv2d
from robustpointclouds_amd import _ffi
from robustpointclouds_amd import center_head as ch
from robustpointclouds_amd import dense_bev as db
from robustpointclouds_amd.center_head import _BOX_ORDER, CenterHead
from tests._dense_masks import FlipStats

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


def _bf(t):
    return t.to(torch.bfloat16).to(torch.float64)


def _rel(a, b):
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


@pytest.mark.parametrize("B,H,W,amp", [(2, 16, 24, 0.8), (1, 8, 8, 2.5), (1, 16, 16, 6.0), (2, 16, 24, 0.0)])
def test_dcn_forward_backward_f32(B, H, W, amp):
    """fp32 parity-mode DCN (large offsets in the third case: most corners leave the tile window; amp 0: zero
    offsets and offset bias — upstream's zero-initialised offset convs, every sample exactly on an integer
    position, where mmcv's offset gradient is one-sided and samples at -1 / H carry none)."""
    g = torch.Generator().manual_seed(int(amp * 10) + H + 1)
    x = torch.randn(B, 64, H, W, generator=g).double()
    offz = torch.randn(B, 64, H, W, generator=g).double() * amp
    offz[:, 18:] = 0
    ob = torch.randn(18, generator=g).double() * (0.3 if amp > 0 else 0.0)
    Wt = torch.randn(64, 16, 3, 3, generator=g).double() * 0.1
    gout = torch.randn(B, 64, H, W, generator=g).double()
    x, offz, ob, Wt, gout = (t.float().double() for t in (x, offz, ob, Wt, gout))
    lib = _ffi.load()
    st = _ffi.stream_of(torch.empty(1, device=DEV))
    xi = db._nhwc(x.to(DEV), torch.float32)
    oi = db._nhwc(offz.to(DEV), torch.float32)
    obd = ob.float().to(DEV)
    W32 = Wt.float().to(DEV).contiguous()
    out = db._image(B, 64, H, W, DEV, torch.float32)
    _ffi.check(lib.rpc_dcn_forward_f32(_ffi.ptr(xi), 64, _ffi.ptr(oi), 64, _ffi.ptr(obd), _ffi.ptr(W32),
                                       _ffi.ptr(out), 64, B, H, W, st), "fwd")
    gi = db._nhwc(gout.to(DEV), torch.float32)
    dx = torch.zeros((B * H * W, 64), dtype=torch.float32, device=DEV)
    doff = db._image(B, 64, H, W, DEV, torch.float32)
    dob = torch.empty(18, device=DEV)
    dW = torch.empty((64, 16, 3, 3), device=DEV)
    wsz = lib.rpc_dcn_backward_workspace_size(B, H, W)
    ws = torch.empty(wsz, dtype=torch.uint8, device=DEV)
    _ffi.check(lib.rpc_dcn_backward_f32(_ffi.ptr(xi), 64, _ffi.ptr(oi), 64, _ffi.ptr(obd), _ffi.ptr(W32),
                                        _ffi.ptr(gi), 64, _ffi.ptr(dx), _ffi.ptr(doff), 64, _ffi.ptr(dob),
                                        _ffi.ptr(dW), B, H, W, _ffi.ptr(ws), wsz, st), "bwd")
    xr = x.clone().requires_grad_(True)
    offr = (offz[:, :18] + ob.view(1, 18, 1, 1)).clone().requires_grad_(True)
    Wr = Wt.clone().requires_grad_(True)
    ref = deform_conv2d(xr, offr, Wr, groups=4)
    (ref * gout).sum().backward()
    assert _rel(out.cpu().double(), ref.detach()) <= 1e-5
    assert _rel(dx.view(B, H, W, 64).permute(0, 3, 1, 2).cpu().double(), xr.grad) <= 1e-4
    assert _rel(doff.cpu().double()[:, :18], offr.grad) <= 1e-4
    assert float(doff[:, 18:].abs().max()) == 0.0
    assert _rel(dob.cpu().double(), offr.grad.sum((0, 2, 3))) <= 1e-4
    assert _rel(dW.cpu().double(), Wr.grad) <= 1e-4


@pytest.mark.parametrize("B,H,W,amp", [(2, 16, 24, 0.8), (1, 8, 8, 2.5)])
def test_dcn_forward_backward(B, H, W, amp):
    g = torch.Generator().manual_seed(int(amp * 10) + H)
    x = _bf(torch.randn(B, 64, H, W, generator=g))
    offz = _bf(torch.randn(B, 64, H, W, generator=g) * amp)          # offset-conv output image, 64 wide
    offz[:, 18:] = 0
    ob = torch.randn(18, generator=g).double() * 0.3
    Wt = _bf(torch.randn(64, 16, 3, 3, generator=g) * 0.1)
    gout = _bf(torch.randn(B, 64, H, W, generator=g))
    lib = _ffi.load()
    st = _ffi.stream_of(torch.empty(1, device=DEV))
    xi = db._nhwc(x.float().to(DEV))
    oi = db._nhwc(offz.float().to(DEV))
    obd = ob.float().to(DEV)
    W32 = Wt.float().to(DEV).contiguous()
    wf = torch.empty((9, 64, 64), dtype=torch.bfloat16, device=DEV)
    wd = torch.empty((9, 64, 64), dtype=torch.bfloat16, device=DEV)
    _ffi.check(lib.rpc_dcn_prep_weight(_ffi.ptr(W32), _ffi.ptr(wf), _ffi.ptr(wd), st), "prep")
    out = db._image(B, 64, H, W, DEV)
    _ffi.check(lib.rpc_dcn_forward(_ffi.ptr(xi), 64, _ffi.ptr(oi), 64, _ffi.ptr(obd), _ffi.ptr(wf), _ffi.ptr(out), 64,
                                   B, H, W, st), "fwd")
    gi = db._nhwc(gout.float().to(DEV))
    dx = torch.zeros((B * H * W, 64), dtype=torch.float32, device=DEV)
    doff = db._image(B, 64, H, W, DEV)
    dob = torch.empty(18, device=DEV)
    dW = torch.empty((64, 16, 3, 3), device=DEV)
    wsz = lib.rpc_dcn_backward_workspace_size(B, H, W)
    ws = torch.empty(wsz, dtype=torch.uint8, device=DEV)
    _ffi.check(lib.rpc_dcn_backward(_ffi.ptr(xi), 64, _ffi.ptr(oi), 64, _ffi.ptr(obd), _ffi.ptr(wd), _ffi.ptr(gi), 64,
                                    _ffi.ptr(dx), _ffi.ptr(doff), 64, _ffi.ptr(dob), _ffi.ptr(dW), B, H, W, _ffi.ptr(ws),
                                    wsz, st), "bwd")
    # reference (offsets = bf16 conv output + fp32 bias, as the kernel reads them)
    xr = x.clone().requires_grad_(True)
    offr = (offz[:, :18] + ob.view(1, 18, 1, 1)).clone().requires_grad_(True)
    Wr = Wt.clone().requires_grad_(True)
    ref = deform_conv2d(xr, offr, Wr, groups=4)
    (ref * gout).sum().backward()
    got = out.float().cpu().double()
    assert _rel(got, ref.detach()) <= 1e-2
    assert _rel(dx.view(B, H, W, 64).permute(0, 3, 1, 2).cpu().double(), xr.grad) <= 2e-2
    assert _rel(doff.float().cpu().double()[:, :18], offr.grad) <= 2e-2
    assert float(doff.float()[:, 18:].abs().max()) == 0.0
    assert _rel(dob.cpu().double(), offr.grad.sum((0, 2, 3))) <= 2e-2
    assert _rel(dW.cpu().double(), Wr.grad) <= 2e-2


@pytest.mark.parametrize("f32", [False, True])
def test_dcn_backward_offset_slice(f32):
    """rpc_dcn_backward(_f32)_ex with 18 offset-gradient channels: the DCN reads its offsets from channel 18 j
    of a shared 256-wide image and writes exactly its 18 gradient channels there (the head's concatenated
    offset conv), bit-identical to the 64-wide padded form; the neighbours' channels are untouched."""
    B, H, W, j, P = 2, 16, 24, 5, 256
    dt = torch.float32 if f32 else torch.bfloat16
    g = torch.Generator().manual_seed(11)
    x = torch.randn(B, 64, H, W, generator=g)
    offw = torch.randn(B, P, H, W, generator=g) * 1.5
    ob = (torch.randn(18, generator=g) * 0.3).to(DEV)
    Wt = (torch.randn(64, 16, 3, 3, generator=g) * 0.1).to(DEV).contiguous()
    gout = torch.randn(B, 64, H, W, generator=g)
    lib = _ffi.load()
    st = _ffi.stream_of(torch.empty(1, device=DEV))
    xi, gi = db._nhwc(x.to(DEV), dt), db._nhwc(gout.to(DEV), dt)
    wide = db._nhwc(offw.to(DEV), dt)
    narrow = db._nhwc(torch.cat([offw[:, 18 * j:18 * (j + 1)], torch.zeros(B, 46, H, W)], 1).to(DEV), dt)
    if f32:
        wb = Wt
    else:
        wf = torch.empty((9, 64, 64), dtype=torch.bfloat16, device=DEV)
        wb = torch.empty((9, 64, 64), dtype=torch.bfloat16, device=DEV)
        _ffi.check(lib.rpc_dcn_prep_weight(_ffi.ptr(Wt), _ffi.ptr(wf), _ffi.ptr(wb), st), "prep")
    wsz = lib.rpc_dcn_backward_workspace_size(B, H, W)
    ws = torch.empty(wsz, dtype=torch.uint8, device=DEV)
    res = []
    for mode in ("pad", "slice"):
        dx = torch.zeros((B * H * W, 64), dtype=torch.float32, device=DEV)
        dob = torch.empty(18, device=DEV)
        dW = torch.empty((64, 16, 3, 3), device=DEV)
        if mode == "pad":
            doff = db._image(B, 64, H, W, DEV, dt)
            fn = lib.rpc_dcn_backward_f32_ex if f32 else lib.rpc_dcn_backward_ex
            _ffi.check(fn(_ffi.ptr(xi), 64, _ffi.ptr(narrow), 64, _ffi.ptr(ob), _ffi.ptr(wb), _ffi.ptr(gi), 64,
                          _ffi.ptr(dx), _ffi.ptr(doff), 64, 64, _ffi.ptr(dob), _ffi.ptr(dW), B, H, W, _ffi.ptr(ws), wsz,
                          st), "bwd pad")
            got = doff[:, :18]
        else:
            doff = torch.full((B, H, W, P), 7.0, dtype=dt, device=DEV).permute(0, 3, 1, 2)
            fn = lib.rpc_dcn_backward_f32_ex if f32 else lib.rpc_dcn_backward_ex
            _ffi.check(fn(_ffi.ptr(xi), 64, _ffi.ptr(wide[:, 18 * j:]), P, _ffi.ptr(ob), _ffi.ptr(wb), _ffi.ptr(gi),
                          64, _ffi.ptr(dx), _ffi.ptr(doff[:, 18 * j:]), P, 18, _ffi.ptr(dob), _ffi.ptr(dW), B, H, W,
                          _ffi.ptr(ws), wsz, st), "bwd slice")
            got = doff[:, 18 * j:18 * (j + 1)]
            rest = torch.cat([doff[:, :18 * j], doff[:, 18 * (j + 1):]], 1)
            assert bool((rest == 7.0).all())
        res.append((dx.clone(), got.clone(), dob.clone(), dW.clone()))
    (dx0, *r0), (dx1, *r1) = res
    assert _rel(dx1.double(), dx0.double()) <= 1e-6   # input gradient: float atomics (summation order)
    for a, b in zip(r0, r1):
        assert torch.equal(a, b)
    # argument checks: misaligned slice, unsupported channel count
    bad = db._image(B, P, H, W, DEV, dt)
    fn = lib.rpc_dcn_backward_f32_ex if f32 else lib.rpc_dcn_backward_ex
    assert fn(_ffi.ptr(xi), 64, _ffi.ptr(wide), P, _ffi.ptr(ob), _ffi.ptr(wb), _ffi.ptr(gi), 64, _ffi.ptr(dx),
              _ffi.ptr(bad[:, 1:]), P, 18, _ffi.ptr(dob), _ffi.ptr(dW), B, H, W, _ffi.ptr(ws), wsz, st) != 0
    assert fn(_ffi.ptr(xi), 64, _ffi.ptr(wide), P, _ffi.ptr(ob), _ffi.ptr(wb), _ffi.ptr(gi), 64, _ffi.ptr(dx),
              _ffi.ptr(bad), P, 20, _ffi.ptr(dob), _ffi.ptr(dW), B, H, W, _ffi.ptr(ws), wsz, st) != 0


FLIP_PRE_MAX = 1e-4   # an adopted ReLU decision float64 takes differently lies within this of 0 (x channel max)


def head_masks(trace):
    """center_head.DEBUG -> {ConvModule name: bool mask [B, 64, H, W]}: the engine's ReLU decisions, the sign of
    fmaf(z - mean, scale, beta) recomputed exactly from the stored fp32 values (tests/_dense_masks.engine_masks)."""
    out = {}
    for name, z, bn, sl, B, H, W in trace:
        co = z.shape[1]
        sc, be, mu = bn[:co], bn[co:2 * co], bn[2 * co:3 * co]
        pre = (z.float() - mu.float()).double() * sc.double() + be.double()
        if sl is not None:
            pre = pre[:, sl]
        out[name] = (pre > 0).view(B, H, W, -1).permute(0, 3, 1, 2).contiguous().cpu()
    return out


def _cm_ref(P, prefix, h, masks=None, flips=None):
    """ConvModule (conv, train-mode BatchNorm, ReLU) in float64; with masks, on the engine's ReLU decisions
    (same-branch parity): a pre-activation within an fp32 rounding of 0 lands on either side in fp32, and on
    the other side it moves every gradient below it (r06: 1.5e-3 of the input gradient at zero offsets)."""
    z = Fn.conv2d(h, P[prefix + ".conv.weight"], padding=1)
    m = z.mean((0, 2, 3), keepdim=True)
    v = z.var((0, 2, 3), unbiased=False, keepdim=True)
    pre = (z - m) / torch.sqrt(v + 1e-5) * P[prefix + ".bn.weight"].view(1, -1, 1, 1) + \
        P[prefix + ".bn.bias"].view(1, -1, 1, 1)
    if masks is None:
        return torch.relu(pre)
    mk = masks[prefix]
    if flips is not None:
        a = pre.detach()
        d = mk != (a > 0)
        if bool(d.any()):
            sc = a.abs().amax(dim=(0, 2, 3), keepdim=True).clamp_min(1e-30)
            flips.flips += int(d.sum())
            flips.worst = max(flips.worst, float((a.abs() / sc)[d].max()))
    return pre * mk.to(pre.dtype)


def _ref_head(head, x, B, H, W, masks=None, flips=None):
    """float64 torch forward of the same stack (BN in training mode: batch statistics)."""
    P = {k: v.detach().cpu().double() for k, v in head.named_parameters()}

    def cm(prefix, h):
        return _cm_ref(P, prefix, h, masks, flips)

    def fc(prefix, h):
        return Fn.conv2d(h, P[prefix + ".weight"], P[prefix + ".bias"], padding=1)

    y0 = cm("shared_conv", x)
    hms, boxes = [], []
    for t, th in enumerate(head.task_heads):
        feats = {}
        for br in ("cls", "reg"):
            pre = f"task_heads.{t}.feature_adapt_{br}"
            off = Fn.conv2d(y0, P[pre + ".conv_offset.weight"], P[pre + ".conv_offset.bias"], padding=1)
            feats[br] = deform_conv2d(y0, off, P[pre + ".weight"], groups=4)
        hms.append(fc(f"task_heads.{t}.cls_head.1", cm(f"task_heads.{t}.cls_head.0", feats["cls"])))
        boxes.append(torch.cat([fc(f"task_heads.{t}.task_head.{n}.1", cm(f"task_heads.{t}.task_head.{n}.0",
                                                                           feats["reg"])) for n in _BOX_ORDER], 1))
    return torch.cat(hms, 1), torch.cat(boxes, 1), P


@pytest.mark.parametrize("offsets", ["random", "zero"])
@pytest.mark.parametrize("mode", ["bf16", "fp32"])
def test_center_head_forward_backward(mode, offsets):
    """offsets "random": offset convs drawn so the samples spread over whole cells; "zero": upstream's own starting
    state — the DCNSeparateHead offset convs are zero-initialised, so every sample lies exactly ON an integer
    position (a cell edge), where mmcv's offset gradient is one-sided (get_coordinate_weight on the cell
    [floor(p), floor(p) + 1]; samples at p = -1 or p = H lie outside and carry none). The offset-conv gradients
    are then the whole learning signal of the DCN offsets in the reference's first step."""
    f32 = mode == "fp32"
    tol_out, tol_x, cos_min = (1e-4, 1e-3, 0.99999) if f32 else (3e-2, None, 0.98)
    torch.manual_seed(0)
    B, Cin, H, W = 2, 128, 32, 32
    head = CenterHead(in_channels=Cin).to(DEV)
    if offsets == "zero":
        for th in head.task_heads:   # (the constructor's own init, asserted)
            for dcn in (th.feature_adapt_cls, th.feature_adapt_reg):
                assert float(dcn.conv_offset.weight.abs().max()) == 0.0
                assert float(dcn.conv_offset.bias.abs().max()) == 0.0
    else:
        with torch.no_grad():   # non-zero offsets (the offset convs are zero-initialised)
            for th in head.task_heads:
                for dcn in (th.feature_adapt_cls, th.feature_adapt_reg):
                    dcn.conv_offset.weight.normal_(0, 0.05)
                    dcn.conv_offset.bias.uniform_(-0.5, 0.5)
    x = _bf(torch.randn(B, Cin, H, W)).float()
    xd = x.to(DEV).to(torch.float32 if f32 else torch.bfloat16).requires_grad_(True)
    ch.DEBUG = [] if f32 else None
    try:
        preds = head([xd])
        masks = head_masks(ch.DEBUG) if f32 else None
    finally:
        ch.DEBUG = None
    hm = torch.cat([p[0]["heatmap"] for p in preds], 1)
    box = torch.cat([torch.cat([p[0][n] for n in _BOX_ORDER], 1) for p in preds], 1)
    xr = x.double().requires_grad_(True)
    # fp32: the float64 reference on the engine's ReLU decisions (same-branch parity), every decision it would
    # take differently within FLIP_PRE_MAX of zero; bf16: its own decisions (direction-level bounds)
    flips = FlipStats()
    rhm, rbox, _ = _ref_head(head, xr, B, H, W, masks, flips)
    print(f"{mode}-{offsets}: ReLU decisions differing from float64's: {flips}")
    assert flips.worst <= FLIP_PRE_MAX, flips
    assert _rel(hm.detach().cpu().double(), rhm.detach()) <= tol_out
    assert _rel(box.detach().cpu().double(), rbox.detach()) <= tol_out
    g = torch.Generator().manual_seed(5)
    ghm, gbox = torch.randn(rhm.shape, generator=g).double(), torch.randn(rbox.shape, generator=g).double()
    ((hm * ghm.float().to(DEV)).sum() + (box * gbox.float().to(DEV)).sum()).backward()
    ((rhm * ghm).sum() + (rbox * gbox).sum()).backward()
    cos = lambda a, b: (a.flatten() @ b.flatten() / (a.norm() * b.norm())).item()
    ex = _rel(xd.grad.cpu().double(), xr.grad)
    print(f"{mode}-{offsets}: outputs {_rel(hm.detach().cpu().double(), rhm.detach()):.2e} / "
          f"{_rel(box.detach().cpu().double(), rbox.detach()):.2e}, input gradient {ex:.2e}")
    assert cos(xd.grad.cpu().double(), xr.grad) >= cos_min
    if f32:
        assert ex <= tol_x, ex
    Pref = {}
    P = {k: v.detach().cpu().double().requires_grad_(True) for k, v in head.named_parameters()}
    # parameter gradients: recompute the reference with parameters as leaves
    def cm(prefix, h):
        return _cm_ref(P, prefix, h, masks)
    y0 = cm("shared_conv", x.double())
    tot = 0
    for t, th in enumerate(head.task_heads):
        feats = {}
        for br in ("cls", "reg"):
            pre = f"task_heads.{t}.feature_adapt_{br}"
            off = Fn.conv2d(y0, P[pre + ".conv_offset.weight"], P[pre + ".conv_offset.bias"], padding=1)
            feats[br] = deform_conv2d(y0, off, P[pre + ".weight"], groups=4)
        tot = tot + (Fn.conv2d(cm(f"task_heads.{t}.cls_head.0", feats["cls"]), P[f"task_heads.{t}.cls_head.1.weight"],
                               P[f"task_heads.{t}.cls_head.1.bias"], padding=1) *
                     ghm[:, sum(head.num_classes[:t]):sum(head.num_classes[:t + 1])]).sum()
        bo = 10 * t
        for n, w in zip(_BOX_ORDER, (2, 1, 3, 2, 2)):
            pre = f"task_heads.{t}.task_head.{n}"
            tot = tot + (Fn.conv2d(cm(pre + ".0", feats["reg"]), P[pre + ".1.weight"], P[pre + ".1.bias"], padding=1)
                         * gbox[:, bo:bo + w]).sum()
            bo += w
    tot.backward()
    bad = []
    for k, p in head.named_parameters():
        c = cos(p.grad.cpu().double(), P[k].grad)
        print(f"  {k:48s} rel {_rel(p.grad.cpu().double(), P[k].grad):.2e} cos {c:.6f}")
        if not c >= cos_min or (f32 and not _rel(p.grad.cpu().double(), P[k].grad) <= 5e-3):
            bad.append((k, c, _rel(p.grad.cpu().double(), P[k].grad)))
    assert not bad, bad
