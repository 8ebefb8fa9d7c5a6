"""Dense BEV backbone + neck on the HIP implicit-GEMM engine (perf mode).

`SECOND` (upstream mmdet3d backbones/second.py) and `SECONDFPN` (necks/second_fpn.py), as
configured at configs/adversarial/adversarial-second_hv_secfpn_8xb6-80e_kitti-3d-car.py (base
second_hv_secfpn_kitti.py) and called at models/detectors/adversarial_voxelnet.py:142-145, each
become ONE autograd node over csrc/dense_conv.hip (C-ABI `rpc_dense_*`):

  forward, per Conv-BN-ReLU layer: rpc_dense_conv (bf16 MFMA, NHWC, BatchNorm partial sums in
  the epilogue) -> rpc_bn_finalize (batch statistics, running stats, momentum/eps of the module)
  -> rpc_dense_bn_apply (normalise + ReLU -> bf16 image, the FPN concat written in place)
  backward, per layer: rpc_dense_bnbwd_stats -> rpc_bn_finalize(mode 1) (dgamma, dbeta) ->
  rpc_dense_bnbwd_apply (dz) -> rpc_dense_wgrad (dW, fp32) -> rpc_dense_conv (data gradient:
  flipped-tap S1, D2 for the stride-2 layer, P1 / G2 for the deconvolutions)

Perf mode: activations bf16 channels_last (fp32 accumulation, fp32 BatchNorm statistics); weights
stay fp32 master copies (cast to bf16 GEMM operands per step). Parity mode (fp32 input): the same
node over the fp32 engine (csrc/dense_f32.hip, `rpc_dense_*_f32`: fp32 operands on fp32 MFMA,
fp32 NHWC images) — the engine follows the dtype of the image handed in. The module parameters
and state-dict keys are the torch modules' own (second.py).
"""
from __future__ import annotations

import os
import weakref

import torch

from . import _ffi

S1, S2, D2, P1, U2, G2 = 0, 1, 2, 3, 4, 5


class ConvTimer:
    """HIP-event timing of the S1 (3x3 stride-1: kernels `rpc::dn::k_conv3x3<0>`, `k_conv3x3w<0>`,
    `k_conv3x3x<0>`, `k_conv3x3y<0>`) launches of rpc_dense_conv — forward and flipped-tap data gradient —
    on the stream they are launched on. Algorithmic work per launch = 2 * B*H*W * C_in * C_out * 9 FLOP
    (every tap of a zero-padded 3x3 convolution); algorithmic bytes = bf16 source image + bf16 output
    image + bf16 weights. Data gradients issued through rpc_dense_conv_bnbwd (the same kernel, whose
    epilogue also reads the next layer's pre-activation image for its BatchNorm-backward sums: + one bf16
    image of bytes) are reported as their own entry, "<kernel> +bnbwd".
    bench.py installs one as `dense_bev.TIMER`. Timing events cannot be recorded inside a captured HIP
    graph on ROCm (torch refuses external events), so launches issued during a capture are not timed:
    bench.py times eager steps (graphs off) right after its timed loop — the same kernels and shapes."""

    def __init__(self):
        self.recs = []
        self.enabled = False

    def start(self):
        e = torch.cuda.Event(enable_timing=True)
        e.record(torch.cuda.current_stream())
        return e

    KERNELS = {0: "rpc::dn::k_conv3x3<0>", 1: "rpc::dn::k_conv3x3w<0>", 2: "rpc::dn::k_conv3x3x<0>",
               3: "rpc::dn::k_conv3x3y<0>", 12: "rpc::dn::k_conv3x3x<0> +bnbwd", 13: "rpc::dn::k_conv3x3y<0> +bnbwd"}
    FUSED = 10   # variant offset of the rpc_dense_conv_bnbwd launches

    def stop(self, e0, rows, ci, co, variant=0):
        e1 = torch.cuda.Event(enable_timing=True)
        e1.record(torch.cuda.current_stream())
        self.recs.append((e0, e1, rows, ci, co, variant))

    def reset(self):
        self.recs = []

    @staticmethod
    def _stats(recs, kernel):
        ms = sum(a.elapsed_time(b) for a, b, *_ in recs)
        flops = sum(2.0 * r * ci * co * 9 for _, _, r, ci, co, _v in recs)
        byts = sum(2.0 * r * (ci + co) + 2.0 * 9 * ci * co + (2.0 * r * co if _v >= ConvTimer.FUSED else 0.0)
                   for _, _, r, ci, co, _v in recs)
        n = len(recs)
        return dict(launches=n, avg_ms=ms / n, flops_per_launch=flops / n, bytes_per_launch=byts / n,
                    tflops=flops / (ms * 1e-3) / 1e12, gbps=byts / (ms * 1e-3) / 1e9, kernel=kernel, dtype="bf16",
                    total_ms=ms)

    def summary(self):
        """Per kernel: {kernel name: stats}, each over that kernel's own launches, FLOPs and bytes."""
        torch.cuda.synchronize()
        if not self.recs:
            return None
        out = {}
        for v, name in self.KERNELS.items():
            rs = [r for r in self.recs if r[5] == v]
            if rs:
                out[name] = self._stats(rs, name)
        return out


TIMER = None
# parity tests: a list -> every training forward appends (bn module, z [Mo][co], bn [4co], B, Ho, Wo) per
# layer (the stored pre-BatchNorm image and its scale/beta/mean/invstd: the engine's ReLU decisions)
DEBUG = None

# ---- HIP graphs over the fixed-shape dense part. The SECOND / SECONDFPN forward and backward issue
# ~100 launches per step from Python (weight prep, conv, BN finalize / apply, wgrad, dgrad) with fixed
# shapes for a fixed batch; on a slow host that issue time made the whole step host-bound (r01: one box
# at 553.6 instead of ~720 frames/s with unchanged kernel time). Each autograd node (BackboneFn,
# NeckFn, and their backward) runs eagerly the first time it sees a shape, is captured into a HIP graph
# the second time and replayed afterwards: inputs are copied into the captured static inputs only when
# the caller passes other storage (the FPN reads the backbone graph's own outputs in place), outputs
# are the graph's static tensors (overwritten by the next replay, after this step has consumed them).
# RPC_DENSE_GRAPHS=0 turns it off.
GRAPHS = os.environ.get("RPC_DENSE_GRAPHS", "1") != "0"
_CAPTURING = [False]


def _capturing() -> bool:
    return _CAPTURING[0]


class _GraphEntry:
    def __init__(self):
        self.calls = 0
        self.graph = None
        self.static_in = None
        self.outs = None
        self.state = None
        self.bwd = {}


# data_ptr -> tensor: storage that stays put across steps (graph outputs, persistent buffers). Weak:
# an entry lives only as long as its owner keeps the tensor (a graph entry, a module's buffer cache)
_STABLE = weakref.WeakValueDictionary()


def mark_stable(t: torch.Tensor) -> None:
    """Declare `t`'s storage persistent (reused, never freed, by its owner across steps): a graph
    captured with it as an input reads it in place instead of from a copy."""
    _STABLE[t.data_ptr()] = t


# data_ptr -> tensor: persistent gradient images owned by a module's graph cache (the FPN's data
# gradients): rewritten every step before they are read, so a consumer may add into them
_SCRATCH = weakref.WeakValueDictionary()


class _GraphCache(dict):
    """A module's HIP graph entries and persistent images, kept in the module's own __dict__ so they
    are freed with it (a module-level cache keyed by id(module) could hand a new module that reuses
    the id a stale graph). Not copied by deepcopy / pickling: a copy captures its own graphs."""

    def __deepcopy__(self, memo):
        return _GraphCache()

    def __reduce__(self):
        return (_GraphCache, ())


def graph_cache(mod) -> "_GraphCache":
    c = mod.__dict__.get("_hip_graphs")
    if c is None:
        c = mod.__dict__["_hip_graphs"] = _GraphCache()
    return c


def _state_key(mod):
    """Addresses the captured kernels read and write (weights, BN affine, running statistics): a
    replaced or moved parameter / buffer forces a new capture instead of a replay of stale pointers."""
    return tuple(t.data_ptr() for t in mod.parameters()) + tuple(t.data_ptr() for t in mod.buffers())


def _scratch_image(cache, key, B, C, H, W, dev, dt):
    """A persistent NHWC image for `key` in a module's graph cache (stable: the backbone's backward
    graph reads it in place)."""
    t = cache.get(key)
    if t is None:
        t = _image(B, C, H, W, dev, dt)
        cache[key] = t
        _SCRATCH[t.data_ptr()] = t
        mark_stable(t)
    return t


def _static_in(t):
    if t is None:
        return None
    if t.data_ptr() in _STABLE:
        return t
    s_ = torch.empty_strided(t.size(), t.stride(), dtype=t.dtype, device=t.device)
    s_.copy_(t)
    return s_


def _graph_run(cache, key, inputs, body, eager_first=True):
    """body(*inputs) -> (outputs, state): eager on the first call for `key` (eager_first), captured
    into a HIP graph on the next one and replayed from then on. Returns (outputs, state, entry)."""
    e = cache.get(key)
    if e is None:
        e = cache[key] = _GraphEntry()
    e.calls += 1
    if eager_first and e.calls == 1:
        outs, state = body(*inputs)
        return outs, state, None
    if e.graph is None:
        e.static_in = [_static_in(t) for t in inputs]
        g = torch.cuda.CUDAGraph()
        _CAPTURING[0] = True
        try:
            with torch.cuda.graph(g, capture_error_mode="thread_local"):
                e.outs, e.state = body(*e.static_in)
        finally:
            _CAPTURING[0] = False
        e.graph = g
        for o in (e.outs if isinstance(e.outs, (tuple, list)) else (e.outs,)):
            if isinstance(o, torch.Tensor):
                mark_stable(o)
    else:
        for s_, t in zip(e.static_in, inputs):
            if t is not None and s_.data_ptr() != t.data_ptr():
                s_.copy_(t)
    e.graph.replay()
    return e.outs, e.state, e


def _conv(lib, fmap, *args):
    """rpc_dense_conv, with the S1 launches timed when a ConvTimer is enabled."""
    t = TIMER if (TIMER is not None and TIMER.enabled and not _capturing() and fmap == S1 and args[4] % 128 == 0) \
        else None
    e0 = t.start() if t is not None else None
    rc = lib.rpc_dense_conv(fmap, *args)
    if t is not None:
        r = _ffi_img_rows(args[10])
        t.stop(e0, r, args[2], args[4], lib.rpc_dense_conv_s1_kernel(fmap, args[4], args[10]))
    return rc


RPC_ERR_UNSUPPORTED = 3
# S1 data gradients write the BatchNorm-backward sums of the layer they feed (A/B: RPC_DENSE_BNFUSE=0)
BN_FUSE = os.environ.get("RPC_DENSE_BNFUSE", "1") != "0"


def _conv_bnbwd(lib, *args):
    """rpc_dense_conv_bnbwd (an S1 data gradient + the BatchNorm-backward sums of the layer it enters), timed
    like _conv's S1 launches when a ConvTimer is enabled. Returns the rpc status."""
    t = TIMER if (TIMER is not None and TIMER.enabled and not _capturing() and args[4] % 128 == 0) else None
    e0 = t.start() if t is not None else None
    rc = lib.rpc_dense_conv_bnbwd(*args)
    if t is not None and rc == 0:
        r = _ffi_img_rows(args[10])
        t.stop(e0, r, args[2], args[4], ConvTimer.FUSED + lib.rpc_dense_conv_s1_kernel(S1, args[4], args[10]))
    return rc


def _ffi_img_rows(arr):
    return int(arr[0]) * int(arr[1]) * int(arr[2])


def _nhwc(t: torch.Tensor, dt=torch.bfloat16) -> torch.Tensor:
    """[B, C, H, W] -> a channels_last tensor of dtype dt (its storage is the NHWC image)."""
    t = t.to(dt)
    if not t.is_contiguous(memory_format=torch.channels_last):
        t = t.contiguous(memory_format=torch.channels_last)
    return t


def _image(B, C, H, W, dev, dt=torch.bfloat16):
    return torch.empty((B, H, W, C), dtype=dt, device=dev).permute(0, 3, 1, 2)


class _Eng:
    """The C-ABI entry points of one engine: bf16 (perf mode) or fp32 (parity mode)."""

    def __init__(self, lib, f32: bool):
        self.f32 = f32
        self.dt = torch.float32 if f32 else torch.bfloat16
        x = "_f32" if f32 else ""
        self.conv_raw = getattr(lib, "rpc_dense_conv" + x)
        self.blocks = getattr(lib, "rpc_dense_conv_blocks" + x)
        # BatchNorm partial-sum rows one conv writes (bf16 S1: one per 16x32 tile)
        self.part_rows = (lambda fmap, co, ri: self.blocks(fmap, ri)) if f32 else \
            (lambda fmap, co, ri: lib.rpc_dense_conv_part_rows(fmap, co, ri))
        self.wgrad = getattr(lib, "rpc_dense_wgrad" + x)
        self.wgrad_ws = getattr(lib, "rpc_dense_wgrad_workspace_size" + x)
        self.bn_apply = getattr(lib, "rpc_dense_bn_apply" + x)
        self.bnbwd_stats = getattr(lib, "rpc_dense_bnbwd_stats" + x)
        self.bnbwd_apply = getattr(lib, "rpc_dense_bnbwd_apply" + x)
        self.wprep_batch = getattr(lib, "rpc_dense_wprep_batch" + x)
        self.lib = lib

    def conv(self, fmap, *args):
        if self.f32:
            return self.conv_raw(fmap, *args)
        return _conv(self.lib, fmap, *args)

    def check_widths(self, layers):
        for L in layers:
            if self.f32:
                if L.ci % 16 or L.co % 64:
                    raise RuntimeError(f"fp32 HIP dense conv needs C_in % 16 == 0 and C_out % 64 == 0 "
                                       f"(got {L.ci}->{L.co})")
            elif L.ci % 128 or L.co % 128:
                raise RuntimeError(f"HIP dense conv needs channel counts that are multiples of 128 (got {L.ci}->{L.co})")


def _engine(lib, t: torch.Tensor) -> _Eng:
    if not t.is_cuda:
        raise RuntimeError("the dense BEV engine runs on the HIP kernels only: got a CPU tensor")
    if t.dtype not in (torch.float32, torch.bfloat16):
        raise RuntimeError(f"dense BEV engine: fp32 (parity) or bf16 (perf) images, got {t.dtype}")
    return _Eng(lib, t.dtype == torch.float32)


def _bn_eval(bnm, dev):
    inv = torch.rsqrt(bnm.running_var.float() + bnm.eps)
    return torch.cat([bnm.weight.float() * inv, bnm.bias.float(), bnm.running_mean.float(), inv]).contiguous()


class _Layer:
    """One Conv/Deconv + BatchNorm2d + ReLU: geometry and the C-ABI calls for it."""

    def __init__(self, fmap, conv, bnm, kind, ci, co, taps):
        self.map, self.conv, self.bnm, self.kind = fmap, conv, bnm, kind
        self.ci, self.co, self.taps = ci, co, taps

    def images(self, B, H, W):
        """(row image, source image, output image, output H, W) of the forward GEMM for input H x W."""
        if self.map == S1 or self.map == P1:
            return (B, H, W), (B, H, W), (B, H, W), H, W
        if self.map == S2:
            Ho, Wo = (H - 1) // 2 + 1, (W - 1) // 2 + 1
            return (B, Ho, Wo), (B, H, W), (B, Ho, Wo), Ho, Wo
        # U2: rows = input pixels, output = 2x upsampled image
        return (B, H, W), (B, H, W), (B, 2 * H, 2 * W), 2 * H, 2 * W

    def dgrad_map(self):
        return {S1: S1, S2: D2, P1: P1, U2: G2}[self.map]


def _prep_weights(eng, layers, dev, st):
    """GEMM operands (forward [T][co][ci], data gradient [T][ci][co]; bf16 or fp32 by engine) of every
    layer of a module from the fp32 master weights, in one rpc_dense_wprep_batch(_f32) launch."""
    out = []
    for g0 in range(0, len(layers), 16):   # the kernel takes up to 16 layers per launch
        group = layers[g0:g0 + 16]
        descs = (_ffi.RpcDenseWprep * len(group))()
        keep = []   # fp32 copies stay referenced until the launch is enqueued (stream order after that)
        for i, L in enumerate(group):
            W32 = L.conv.weight.detach().float().contiguous()
            keep.append(W32)
            wf = torch.empty((L.taps, L.co, L.ci), dtype=eng.dt, device=dev)
            wd = torch.empty((L.taps, L.ci, L.co), dtype=eng.dt, device=dev)
            descs[i] = _ffi.RpcDenseWprep(W32.data_ptr(), wf.data_ptr(), wd.data_ptr(), L.kind, L.ci, L.co,
                                          L.taps, 1 if L.map == S1 else 0)
            out.append((wf, wd))
        _ffi.check(eng.wprep_batch(descs, len(group), st), "rpc_dense_wprep_batch")
    return out


def _forward_layer(eng, L, h, pitch, B, H, W, training, dev, st, out=None, out_pitch=None, out_off=0, wts=None):
    """z = conv(h); BN (batch or running stats); y = relu(bn(z)) -> (y image, record).
    wts: (forward, data-gradient) bf16 operands from _prep_weights, else prepared here."""
    R, S, O, Ho, Wo = L.images(B, H, W)
    lib = eng.lib
    if wts is None:
        wts = _prep_weights(eng, [L], dev, st)[0]
    wf, wd = wts
    Mo = B * Ho * Wo
    z = torch.empty((Mo, L.co), dtype=eng.dt, device=dev)
    ri, si, oi = _ffi.int_arr(R), _ffi.int_arr(S), _ffi.int_arr(O)
    part = None
    if training:
        nblk = eng.part_rows(L.map, L.co, ri)
        part = torch.empty((nblk, 2 * L.co), dtype=torch.float32, device=dev)
    _ffi.check(eng.conv(L.map, _ffi.ptr(h), pitch, L.ci, _ffi.ptr(wf), L.co, _ffi.ptr(z), L.co, 0, 0,
                        _ffi.ptr(part), ri, si, oi, st), "rpc_dense_conv")
    bnm = L.bnm
    if training:
        bn = torch.empty(4 * L.co, dtype=torch.float32, device=dev)
        _ffi.check(lib.rpc_bn_finalize(_ffi.ptr(part), part.shape[0], L.co, Mo, 0, _ffi.ptr(bnm.weight),
                                       _ffi.ptr(bnm.bias), float(bnm.eps), float(bnm.momentum),
                                       _ffi.ptr(bnm.running_mean), _ffi.ptr(bnm.running_var), None, _ffi.ptr(bn),
                                       None, None, None, st), "rpc_bn_finalize")
    else:
        bn = _bn_eval(bnm, dev)
    if out is None:
        y = _image(B, L.co, Ho, Wo, dev, eng.dt)
        out_pitch, out_off = L.co, 0
    else:
        y = out
    _ffi.check(eng.bn_apply(_ffi.ptr(z), Mo, L.co, _ffi.ptr(bn), _ffi.ptr(y), out_pitch, out_off, st),
               "rpc_dense_bn_apply")
    rec = dict(L=L, h=h, pitch=pitch, z=z, bn=bn, wd=wd, R=R, S=S, O=O, in_hw=(H, W), Mo=Mo, out_bhw=(B, Ho, Wo))
    return y, rec, Ho, Wo


# (r04 measured the SECOND backbone's weight gradients on a side stream beside the data-gradient chain:
# slower — SECOND 835.8 / 827.8 -> 766.0 / 627.2 frames/s, profiles/r04_ab_dense_wg_side.txt — and r05
# removed it: they run on the training stream.)


def _backward_layer(eng, rec, dh, dh_pitch, dh_off, dev, st, need_dx, dx_out=None, accumulate=False,
                    bn_part=None, next_rec=None):
    """BN+ReLU backward, weight gradient and (optionally) data gradient of one layer.
    bn_part: this layer's BatchNorm-backward partial sums, already written by the data-gradient conv that
    produced dh (rpc_dense_conv_bnbwd) — else rpc_dense_bnbwd_stats computes them. next_rec: the layer the
    data gradient dx enters (its BN + ReLU backward is next): an S1 bf16 data gradient then writes that
    layer's partial sums too, returned as the 5th value (None when not fused)."""
    lib = eng.lib
    L = rec["L"]
    Mo, co, ci = rec["Mo"], L.co, L.ci
    if bn_part is not None:
        part = bn_part
        nb = part.shape[0]
    else:
        nb = lib.rpc_dense_bnbwd_blocks(Mo)
        # the fp32 (parity) engine sums in double (sparse BEV images: the sums cancel)
        part = torch.empty((nb, 2 * co), dtype=torch.float64 if eng.f32 else torch.float32, device=dev)
        _ffi.check(eng.bnbwd_stats(_ffi.ptr(dh), dh_pitch, dh_off, _ffi.ptr(rec["z"]), Mo, co,
                                   _ffi.ptr(rec["bn"]), _ffi.ptr(part), st), "rpc_dense_bnbwd_stats")
    bnb = torch.empty(5 * co, dtype=torch.float32, device=dev)
    dgamma = torch.empty(co, dtype=torch.float32, device=dev)
    dbeta = torch.empty(co, dtype=torch.float32, device=dev)
    mode = 1 | (4 if part.dtype == torch.float64 else 0)   # RPC_BN_PART_F64
    _ffi.check(lib.rpc_bn_finalize(_ffi.ptr(part), nb, co, Mo, mode, _ffi.ptr(L.bnm.weight), _ffi.ptr(L.bnm.bias),
                                   0.0, 0.0, None, None, _ffi.ptr(rec["bn"]), _ffi.ptr(bnb), _ffi.ptr(dgamma),
                                   _ffi.ptr(dbeta), None, st), "rpc_bn_finalize(bwd)")
    dz = torch.empty((Mo, co), dtype=eng.dt, device=dev)
    _ffi.check(eng.bnbwd_apply(_ffi.ptr(dh), dh_pitch, dh_off, _ffi.ptr(rec["z"]), Mo, co,
                                         _ffi.ptr(rec["bn"]), _ffi.ptr(bnb), _ffi.ptr(dz), st),
               "rpc_dense_bnbwd_apply")
    ri, si, oi = _ffi.int_arr(rec["R"]), _ffi.int_arr(rec["S"]), _ffi.int_arr(rec["O"])
    # torch-contiguous layout (the kernel writes [co][ci][kh][kw] / [ci][co][kh][kw] densely), even when
    # the module was converted to channels_last
    dW = torch.empty(tuple(L.conv.weight.shape), dtype=torch.float32, device=dev)
    wsz = eng.wgrad_ws(L.map, ri, ci, co)
    ws = _ffi.workspace(wsz, dev)
    # the U2 weight-gradient GEMM reads dz at the output rows; the others read it at the GEMM rows
    _ffi.check(eng.wgrad(L.map, L.kind, _ffi.ptr(rec["h"]), rec["pitch"], ci, _ffi.ptr(dz), co, co,
                                   ri, si, oi, _ffi.ptr(dW), _ffi.ptr(ws), wsz, st), "rpc_dense_wgrad")
    dx = None
    next_part = None
    if need_dx:
        dmap = L.dgrad_map()
        B, H, W = rec["S"]
        dx = dx_out if dx_out is not None else _image(B, ci, H, W, dev, eng.dt)
        # data gradient GEMM: rows = forward source pixels, source image = forward output image
        if L.map == U2:
            rd, sd = rec["R"], rec["O"]
        else:
            rd, sd = rec["S"], rec["O"]
        rc = None
        if (BN_FUSE and next_rec is not None and not eng.f32 and dmap == S1 and not accumulate and
                next_rec["L"].co == ci):
            ri_d = _ffi.int_arr(rd)
            next_part = torch.empty((lib.rpc_dense_conv_part_rows(S1, ci, ri_d), 2 * ci), dtype=torch.float32,
                                    device=dev)
            rc = _conv_bnbwd(lib, _ffi.ptr(dz), co, co, _ffi.ptr(rec["wd"]), ci, _ffi.ptr(dx), ci,
                             _ffi.ptr(next_rec["z"]), _ffi.ptr(next_rec["bn"]), _ffi.ptr(next_part), ri_d, st)
            if rc == RPC_ERR_UNSUPPORTED:
                next_part = None
            else:
                _ffi.check(rc, "rpc_dense_conv_bnbwd")
        if next_part is None:
            _ffi.check(eng.conv(dmap, _ffi.ptr(dz), co, co, _ffi.ptr(rec["wd"]), ci, _ffi.ptr(dx), ci, 0,
                                1 if accumulate else 0, None, _ffi.int_arr(rd), _ffi.int_arr(sd),
                                _ffi.int_arr(rd), st), "rpc_dense_conv(dgrad)")
    return dx, dW, dgamma, dbeta, next_part


def second_layers(mod):
    """_Layer list per block of a SECOND module (Conv2d 3x3 + BN + ReLU sequences)."""
    blocks = []
    for blk in mod.blocks:
        mods = list(blk.children())
        layers = []
        for i in range(0, len(mods), 3):
            conv, bnm = mods[i], mods[i + 1]
            fmap = S2 if conv.stride[0] == 2 else S1
            layers.append(_Layer(fmap, conv, bnm, 0, conv.in_channels, conv.out_channels, 9))
        blocks.append(layers)
    return blocks


def fpn_layers(mod):
    out = []
    for d in mod.deblocks:
        up, bnm = d[0], d[1]
        k = up.kernel_size[0]
        if type(up) is torch.nn.Conv2d and k == 1 and up.stride[0] == 1:   # use_conv_for_no_stride
            out.append(_Layer(P1, up, bnm, 0, up.in_channels, up.out_channels, 1))
            continue
        assert isinstance(up, torch.nn.ConvTranspose2d) and up.stride[0] == k and k in (1, 2), \
            "HIP SECONDFPN supports ConvTranspose2d deblocks with kernel = stride in {1, 2}"
        out.append(_Layer(P1 if k == 1 else U2, up, bnm, 1, up.in_channels, up.out_channels, k * k))
    return out


def _backbone_fwd(eng, mod, x):
    dev = x.device
    st = _ffi.stream_of(x)
    blocks = second_layers(mod)
    xi = _nhwc(x, eng.dt)
    B, C, H, W = xi.shape
    h, pitch = xi, C
    recs, outs = [], []
    wts = iter(_prep_weights(eng, [L for layers in blocks for L in layers], dev, st))
    for layers in blocks:
        brecs = []
        for L in layers:
            h, rec, H, W = _forward_layer(eng, L, h, pitch, B, H, W, mod.training, dev, st, wts=next(wts))
            pitch = L.co
            brecs.append(rec)
        recs.append(brecs)
        outs.append(h)
    if mod.training:
        _ffi.bump_batches([L.bnm for b in blocks for L in b])
    return tuple(outs), recs


def _backbone_bwd(eng, recs, params, need_x, gouts):
    dt = eng.dt
    g_any = next(g for g in gouts if g is not None)
    dev = g_any.device
    st = _ffi.stream_of(g_any)
    grads = {}
    nb = len(recs)
    # dh = complete gradient w.r.t. the output of block bi (its own output gradient plus what
    # block bi+1's first data-gradient GEMM accumulated into a copy of it)
    dh = _nhwc(gouts[-1], dt) if gouts[-1] is not None else None
    dx = None
    for bi in range(nb - 1, -1, -1):
        brecs = recs[bi]
        if dh is None:   # nothing flows through this block
            dh = _nhwc(gouts[bi - 1], dt) if bi > 0 and gouts[bi - 1] is not None else None
            continue
        bn_part = None   # the block's last layer: its dh comes from outside the block
        for li in range(len(brecs) - 1, -1, -1):
            rec = brecs[li]
            dx_out, accumulate = None, False
            if li > 0:
                need_dx = True
            elif bi > 0:
                need_dx = True
                if gouts[bi - 1] is not None:
                    go = _nhwc(gouts[bi - 1], dt)
                    # the FPN's persistent data-gradient image is ours to add into (no copy); any other
                    # incoming gradient is cloned first
                    dx_out = go if go.data_ptr() in _SCRATCH else go.clone(memory_format=torch.channels_last)
                    accumulate = True
            else:
                need_dx = need_x
            dh, dW, dgam, dbet, bn_part = _backward_layer(eng, rec, dh, rec["L"].co, 0, dev, st, need_dx, dx_out,
                                                          accumulate, bn_part=bn_part,
                                                          next_rec=brecs[li - 1] if li > 0 else None)
            grads[id(rec["L"].conv.weight)] = dW
            grads[id(rec["L"].bnm.weight)] = dgam
            grads[id(rec["L"].bnm.bias)] = dbet
        if bi == 0:
            dx = dh
    return (dx,) + tuple(grads.get(id(p)) for p in params), None


def _debug_trace(recs, training):
    if DEBUG is not None and training:
        DEBUG.extend((r["L"].bnm, r["z"], r["bn"]) + tuple(r["out_bhw"]) for r in recs)


def _alias(t):
    return None if t is None else t.detach()


def _shape_key(ts):
    return tuple(None if t is None else (tuple(t.shape), tuple(t.stride()), t.dtype, t.device) for t in ts)


class BackboneFn(torch.autograd.Function):
    """SECOND forward/backward as one node: x [B, Cin, H, W] -> tuple of block outputs (training
    steps replay HIP graphs after the first, see _graph_run)."""

    @staticmethod
    def forward(ctx, x, mod, *params):
        eng = _engine(_ffi.load(), x)
        for b in second_layers(mod):
            eng.check_widths(b)
        ctx.eng = eng
        ctx.param_list = params
        ctx.entry = None
        if GRAPHS and mod.training:
            key = ("second", eng.f32) + _shape_key([x]) + _state_key(mod)
            outs, recs, ctx.entry = _graph_run(graph_cache(mod), key, [x], lambda xx: _backbone_fwd(eng, mod, xx))
            outs = tuple(_alias(o) for o in outs) if ctx.entry is not None else outs
        else:
            outs, recs = _backbone_fwd(eng, mod, x)
        ctx.recs = recs
        _debug_trace([r for b in recs for r in b], mod.training)
        return outs

    @staticmethod
    def backward(ctx, *gouts):
        eng, recs, params = ctx.eng, ctx.recs, ctx.param_list
        need_x = ctx.needs_input_grad[0]
        if ctx.entry is not None:   # the forward replayed a graph: so does the backward
            key = (need_x,) + _shape_key(gouts)
            res, _, _ = _graph_run(ctx.entry.bwd, key, list(gouts),
                                   lambda *g: _backbone_bwd(eng, recs, params, need_x, g), eager_first=False)
            res = tuple(_alias(t) for t in res)
        else:
            res, _ = _backbone_bwd(eng, recs, params, need_x, gouts)
        ctx.recs = None
        ctx.eng = None
        ctx.entry = None
        return (res[0], None) + tuple(res[1:])


def _neck_fwd(eng, mod, h0, h1):
    dev = h0.device
    st = _ffi.stream_of(h0)
    layers = fpn_layers(mod)
    ins = [_nhwc(h0, eng.dt), _nhwc(h1, eng.dt)]
    B, _, H0, W0 = ins[0].shape
    Ctot = sum(L.co for L in layers)
    out = _image(B, Ctot, H0, W0, dev, eng.dt)
    recs = []
    off = 0
    wts = _prep_weights(eng, layers, dev, st)
    for L, hi, wt in zip(layers, ins, wts):
        _, C, H, W = hi.shape
        _, rec, Ho, Wo = _forward_layer(eng, L, hi, C, B, H, W, mod.training, dev, st, out=out, out_pitch=Ctot,
                                        out_off=off, wts=wt)
        assert (Ho, Wo) == (H0, W0), "FPN deblocks must upsample to the first block's resolution"
        rec["off"] = off
        recs.append(rec)
        off += L.co
    if mod.training:
        _ffi.bump_batches([L.bnm for L in layers])
    return out, (recs, Ctot)


class NeckFn(torch.autograd.Function):
    """SECONDFPN forward/backward as one node: (block outputs) -> [B, sum(out), H0, W0]. The training
    forward replays a HIP graph after the first step (reading the backbone graph's outputs in place);
    the backward stays eager (its input, the head's gradient, is fresh storage every step)."""

    @staticmethod
    def forward(ctx, h0, h1, mod, *params):
        eng = _engine(_ffi.load(), h0)
        eng.check_widths(fpn_layers(mod))
        if GRAPHS and mod.training:
            key = ("fpn", eng.f32) + _shape_key([h0, h1]) + _state_key(mod)
            out, st_, ent = _graph_run(graph_cache(mod), key, [h0, h1], lambda a, b: _neck_fwd(eng, mod, a, b))
            out = _alias(out) if ent is not None else out
        else:
            out, st_ = _neck_fwd(eng, mod, h0, h1)
        ctx.recs, ctx.Ctot = st_
        _debug_trace(ctx.recs, mod.training)
        ctx.eng = eng
        ctx.cache = graph_cache(mod)
        ctx.param_list = params
        return out

    @staticmethod
    def backward(ctx, gout):
        eng = ctx.eng
        dev = gout.device
        st = _ffi.stream_of(gout)
        g = _nhwc(gout, eng.dt)
        grads = {}
        dins = []
        for i, rec in enumerate(ctx.recs):
            L = rec["L"]
            dx_out = None
            if GRAPHS:   # persistent: the backbone's backward graph then reads (and adds into) it in place
                B, H, W = rec["S"]
                dx_out = _scratch_image(ctx.cache, ("fpn_dx", i, B, L.ci, H, W, eng.dt, dev), B, L.ci, H, W,
                                        dev, eng.dt)
            dx, dW, dgam, dbet, _ = _backward_layer(eng, rec, g, ctx.Ctot, rec["off"], dev, st, True, dx_out)
            grads[id(L.conv.weight)] = dW
            grads[id(L.bnm.weight)] = dgam
            grads[id(L.bnm.bias)] = dbet
            dins.append(dx)
        ctx.recs = None
        ctx.eng = None
        ctx.cache = None
        return (dins[0], dins[1], None) + tuple(grads.get(id(p)) for p in ctx.param_list)


def backbone_params(mod):
    ps = []
    for layers in second_layers(mod):
        for L in layers:
            ps += [L.conv.weight, L.bnm.weight, L.bnm.bias]
    return ps


def neck_params(mod):
    ps = []
    for L in fpn_layers(mod):
        ps += [L.conv.weight, L.bnm.weight, L.bnm.bias]
    return ps


def second_forward(mod, x):
    return BackboneFn.apply(x, mod, *backbone_params(mod))


def fpn_forward(mod, xs):
    if len(xs) != 2:
        raise RuntimeError("HIP SECONDFPN path is built for the two-block SECOND of the KITTI configs")
    return [NeckFn.apply(xs[0], xs[1], mod, *neck_params(mod))]
