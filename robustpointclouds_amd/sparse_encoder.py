"""SECOND sparse middle encoder on the HIP kernels.

`SparseEncoder` mirrors upstream mmdet3d `SparseEncoder` (the `middle_encoder` of
configs/adversarial/adversarial-second_hv_secfpn_8xb6-80e_kitti-3d-3class.py:19-23, called
at models/detectors/adversarial_voxelnet.py:141) with its defaults: conv_module blocks,
base_channels 16, output_channels 128, encoder_channels ((16,), (32,32,32), (64,64,64),
(64,64,64)), encoder_paddings ((1,), (1,1,1), (1,1,1), ((0,1,1),1,1)), BatchNorm1d eps 1e-3
momentum 0.01, conv bias off, order conv-norm-act, indice keys subm1..4 / spconv2..4 /
spconv_down2, and the final `.dense()` + view(N, C*D, H, W).

The whole encoder is ONE autograd node: forward builds the rulebooks (four host reads
of output counts, one per strided conv), runs 12 implicit-GEMM convs with BatchNorm
statistics in their epilogues and normalisation+ReLU folded into the next conv's gather;
backward walks the layers in reverse (dense gather, BN backward folded into the dgrad
gather, weight grads as split-K slabs). State-dict keys follow mmdet3d's module names;
conv weights are stored [K, C_in, C_out] (k = (kz*3 + ky)*3 + kx).
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass

import torch
from torch import nn

from . import _ffi, dense_bev, stage_timer


@dataclass
class _Spec:
    kind: str          # 'subm' | 'spconv'
    ci: int
    co: int
    ksize: tuple
    stride: tuple
    pad: tuple
    key: str
    lvl_in: int
    lvl_out: int
    name: str
    res: int = -1       # basicblock conv2: index of the layer whose output is the block identity
    mat: bool = False   # output materialised as rows (a block output, or read as an identity)

    @property
    def K(self):
        return self.ksize[0] * self.ksize[1] * self.ksize[2]


# rulebooks / sparse weight gradients on side streams (SparseEncoder.side_stream)
SIDE_STREAMS = os.environ.get("RPC_SPARSE_STREAMS", "1") != "0"
# the backward as one native call (csrc/sparse_exec.hip rpc_sparse_backward); 0: the per-layer Python loop
NATIVE_BACKWARD = os.environ.get("RPC_SPARSE_NATIVE", "1") != "0"
# BatchNorm finalizes fused into the 16-bit GEMMs that produce their partial sums (rpc_spconv_gemm_bf16_fin:
# data gradients; two-level last-arriving blocks): no standalone rpc_bn_finalize launch in the backward of
# sparse layers 1-11.
# RPC_SPARSE_FUSED_FIN=0: separate finalizes (A/B).
# With an agent-scope release per block (buffer_wbl2: every block wrote back its XCD L2's dirty lines, the
# GEMM's fresh output rows) it was k_gemm_bf16<64,4,0> 41 -> 63 us, <64,4,1> 53 -> 92 us
# (profiles/r04_spgemm_fused_fin.txt); with the hand-off data in sc1 stores and no fence (common.h
# last_block_arrive_lite) the data gradient is 54.2 -> 58.6 us against the 6.4 us rpc_bn_finalize launch it
# removes: SECOND 3-class step within noise (7.155 / 7.157 vs 7.160 / 7.153 ms), CenterPoint 159.7 / 160.0 ->
# 161.0 / 161.1 frames/s with the backward finalizes fused (profiles/r04_ab_fused_fin.txt). The forward's
# measured slower on the metric's step (sparse forward 0.70 -> 0.74 ms) and was removed in r05. Fused and
# separate finalizes give bit-identical results on the metric's encoder (tests/test_gpu_sparse_pipe.py)
FUSED_FINALIZE = os.environ.get("RPC_SPARSE_FUSED_FIN", "1") != "0"
# perf mode forward GEMM operands (gathered rows relu(bn(z)) and forward weight tiles): fp16 (default) or bf16
# (RPC_SPARSE_FWD_BF16=1, A/B). The operand rounding of the forward decides the ReLU masks that every gradient
# passes: with bf16 forward operands the perturber's input gradient is 0.237 rel-L2 from float64, with fp16 0.077
# (cosine 0.972 -> 0.997), the backward's bf16 dz rows alike (oracle/sparse_encoder.py bf16_from emulation,
# tests/test_gpu_sparse_layers.py). fp16 MFMA runs at the bf16 rate; the normalised activations and the
# weights sit far inside its range (the dz rows, which would need loss scaling in fp16, stay bf16)
FWD_FMT = 0 if os.environ.get("RPC_SPARSE_FWD_BF16", "0") != "0" else 1
# (r04's neighbour-mask row order and r05's per-block source-row unions staged in LDS were measured slower on the
# metric's step and removed: profiles/r04_perm_ab.txt, profiles/r05_union_ab.txt)


def _t3(v):
    return tuple(v) if isinstance(v, (tuple, list)) else (v, v, v)


def _conv_out(shape, k, s, p):
    return tuple((shape[a] + 2 * p[a] - (k[a] - 1) - 1) // s[a] + 1 for a in range(3))


class _ConvWeight(nn.Module):
    """Holds the sparse conv weight [K, C_in, C_out] (spconv's module slot '0'), K = kernel offsets
    in (kz, ky, kx) row-major order.

    Checkpoints written by upstream mmdet3d over spconv (the `load_from` SECOND weights of
    configs/adversarial/…-3class.py:168) hold the same key with spconv's own layout; loading
    converts them: spconv 2.x [C_out, kz, ky, kx, C_in] (KRSC) and spconv 1.x [kz, ky, kx, C_in, C_out]
    are both accepted, as is this module's [K, C_in, C_out]."""

    def __init__(self, K, ci, co):
        super().__init__()
        self.weight = nn.Parameter(torch.empty(K, ci, co))
        bound = 1.0 / math.sqrt(ci * K)   # kaiming_uniform(a=sqrt(5)) like torch/spconv convs
        nn.init.uniform_(self.weight, -bound, bound)

    def _load_from_state_dict(self, state_dict, prefix, *args, **kwargs):
        key = prefix + "weight"
        t = state_dict.get(key)
        if t is not None and t.dim() == 5:
            state_dict[key] = spconv_to_kio(t, *self.weight.shape)
        super()._load_from_state_dict(state_dict, prefix, *args, **kwargs)


def spconv_to_kio(t: torch.Tensor, K: int, ci: int, co: int) -> torch.Tensor:
    """A 5-D spconv weight -> [K, C_in, C_out]: spconv 2.x [co, kz, ky, kx, ci] or spconv 1.x
    [kz, ky, kx, ci, co]."""
    s = tuple(t.shape)
    if s[0] == co and s[4] == ci and s[1] * s[2] * s[3] == K:          # spconv 2.x (KRSC)
        return t.permute(1, 2, 3, 4, 0).reshape(K, ci, co).contiguous()
    if s[3] == ci and s[4] == co and s[0] * s[1] * s[2] == K:          # spconv 1.x
        return t.reshape(K, ci, co).contiguous()
    raise RuntimeError(f"sparse conv weight of shape {s} is neither spconv 2.x [{co}, kz, ky, kx, {ci}] nor "
                       f"spconv 1.x [kz, ky, kx, {ci}, {co}] for K = {K}")


class _ConvBN(nn.Sequential):
    def __init__(self, K, ci, co, eps, momentum):
        super().__init__(_ConvWeight(K, ci, co), nn.BatchNorm1d(co, eps=eps, momentum=momentum))


class _BasicBlock(nn.Module):
    """mmdet3d SparseBasicBlock(c, c): conv1 (SubMConv3d) + bn1 + ReLU, conv2 + bn2, + identity, ReLU."""

    def __init__(self, c, eps, momentum):
        super().__init__()
        self.conv1 = _ConvWeight(27, c, c)
        self.bn1 = nn.BatchNorm1d(c, eps=eps, momentum=momentum)
        self.conv2 = _ConvWeight(27, c, c)
        self.bn2 = nn.BatchNorm1d(c, eps=eps, momentum=momentum)


class SparseEncoder(nn.Module):
    def __init__(self, in_channels, sparse_shape, order=("conv", "norm", "act"),
                 norm_cfg=dict(type="BN1d", eps=1e-3, momentum=0.01), base_channels=16, output_channels=128,
                 encoder_channels=((16,), (32, 32, 32), (64, 64, 64), (64, 64, 64)),
                 encoder_paddings=((1,), (1, 1, 1), (1, 1, 1), ((0, 1, 1), 1, 1)), block_type="conv_module",
                 return_middle_feats=False):
        super().__init__()
        if tuple(order) != ("conv", "norm", "act") or block_type not in ("conv_module", "basicblock") \
                or return_middle_feats:
            raise NotImplementedError("conv-norm-act order with conv_module / basicblock blocks is built")
        self.block_type = block_type
        eps = norm_cfg.get("eps", 1e-3)
        mom = norm_cfg.get("momentum", 0.01)
        self.sparse_shape = tuple(int(s) for s in sparse_shape)
        self.in_channels = in_channels
        specs = []
        shapes = [self.sparse_shape]
        specs.append(_Spec("subm", in_channels, base_channels, (3, 3, 3), (1, 1, 1), (1, 1, 1), "subm1", 0, 0,
                           "conv_input"))
        self.conv_input = _ConvBN(27, in_channels, base_channels, eps, mom)
        self.encoder_layers = nn.Module()
        ci = base_channels
        lvl = 0
        nst = len(encoder_channels)
        for i, blocks in enumerate(encoder_channels):
            stage = nn.Module()
            for j, co in enumerate(tuple(blocks)):
                pad = _t3(tuple(encoder_paddings[i])[j])
                if block_type == "basicblock":
                    # upstream make_encoder_layers: a stride-2 SparseConv3d closes every stage but the
                    # last, the other entries are SparseBasicBlock(co, co) (their inputs carry co)
                    if j == len(blocks) - 1 and i != nst - 1:
                        out = _conv_out(shapes[lvl], (3, 3, 3), (2, 2, 2), pad)
                        shapes.append(out)
                        specs.append(_Spec("spconv", ci, co, (3, 3, 3), (2, 2, 2), pad, f"spconv{i + 1}", lvl,
                                           lvl + 1, f"encoder_layers.encoder_layer{i + 1}.{j}", mat=True))
                        stage.add_module(str(j), _ConvBN(27, ci, co, eps, mom))
                        lvl += 1
                    else:
                        if ci != co:
                            raise ValueError("SparseBasicBlock needs equal in/out channels")
                        specs[-1].mat = True            # the block identity
                        specs.append(_Spec("subm", co, co, (3, 3, 3), (1, 1, 1), (1, 1, 1), f"subm{i + 1}", lvl,
                                           lvl, f"encoder_layers.encoder_layer{i + 1}.{j}.conv1"))
                        specs.append(_Spec("subm", co, co, (3, 3, 3), (1, 1, 1), (1, 1, 1), f"subm{i + 1}", lvl,
                                           lvl, f"encoder_layers.encoder_layer{i + 1}.{j}.conv2",
                                           res=len(specs) - 2, mat=True))
                        stage.add_module(str(j), _BasicBlock(co, eps, mom))
                    ci = co
                    continue
                if i != 0 and j == 0:
                    out = _conv_out(shapes[lvl], (3, 3, 3), (2, 2, 2), pad)
                    shapes.append(out)
                    specs.append(_Spec("spconv", ci, co, (3, 3, 3), (2, 2, 2), pad, f"spconv{i + 1}", lvl, lvl + 1,
                                       f"encoder_layers.encoder_layer{i + 1}.{j}"))
                    lvl += 1
                else:
                    specs.append(_Spec("subm", ci, co, (3, 3, 3), (1, 1, 1), pad, f"subm{i + 1}", lvl, lvl,
                                       f"encoder_layers.encoder_layer{i + 1}.{j}"))
                stage.add_module(str(j), _ConvBN(27, ci, co, eps, mom))
                ci = co
            self.encoder_layers.add_module(f"encoder_layer{i + 1}", stage)
        out = _conv_out(shapes[lvl], (3, 1, 1), (2, 1, 1), (0, 0, 0))
        shapes.append(out)
        specs.append(_Spec("spconv", ci, output_channels, (3, 1, 1), (2, 1, 1), (0, 0, 0), "spconv_down2", lvl,
                           lvl + 1, "conv_out"))
        self.conv_out = _ConvBN(3, ci, output_channels, eps, mom)
        self.specs = specs
        self.shapes = shapes
        self.output_channels = output_channels
        self._grids = {}
        self.timer = None   # optional KernelTimer (bench.py roofline), see below
        self.debug = None   # optional list: backward appends (layer, coors, z, dy, bn, out) for diagnostics
        self.flop_probe = None   # optional list: forward appends [(rulebook, C_in, C_out)] per step (bench.py)
        # perf mode: forward / dgrad convs on bf16 MFMA with bf16 gathered rows (fp32 accumulate,
        # fp32 BatchNorm statistics); parity mode (default) is fp32 end to end
        self.bf16 = False
        # dense BEV image: NCHW fp32 (default, = spconv .dense()) or the channels_last / bf16 image
        # the perf mode's NHWC MIOpen convolutions consume without a transpose or a cast
        self.dense_nhwc = False
        self.dense_bf16 = False

    def layers(self):
        """(conv weight module, BatchNorm1d) per spec, in spec order."""
        mods = [(self.conv_input[0], self.conv_input[1])]
        for st in self.encoder_layers.children():
            for m in st.children():
                if isinstance(m, _BasicBlock):
                    mods += [(m.conv1, m.bn1), (m.conv2, m.bn2)]
                else:
                    mods.append((m[0], m[1]))
        mods.append((self.conv_out[0], self.conv_out[1]))
        return mods

    def side_stream(self, name, device):
        """A per-encoder side stream ('rb': rulebooks in the forward, 'wg': weight gradients in the backward);
        RPC_SPARSE_STREAMS=0 puts both back on the current stream (A/B measurement)."""
        if not SIDE_STREAMS:
            return torch.cuda.current_stream(device)
        key = (name, str(device))
        s = self.__dict__.setdefault("_side_streams", {}).get(key)
        if s is None:
            s = self._side_streams[key] = _ffi.side_stream(device)
        return s

    def prepare(self, coors: torch.Tensor, batch_size: int, after=None, consumer=None) -> None:
        """Build every rulebook of a future forward over `coors` now (the trainer's batch prefetch calls
        this during the previous step): the four strided output counts are read here, while the GPU
        still runs the current step's queued work, so the forward that uses them issues its GEMMs
        without a single host read. The forward picks the plan up when it sees the same coordinates."""
        if not coors.is_cuda:
            return
        lib = _ffi.load()
        coors = coors.to(torch.int32).contiguous()
        plan = _RulebookPlan(lib, self, coors, coors.shape[0], int(batch_size), coors.device, after=after,
                             consumer=consumer)
        for li in range(len(self.specs)):
            plan.get(li)
        prepared = self.__dict__.setdefault("_prepared", {})
        while len(prepared) >= 2:          # the batch in flight and the next one; drop older plans
            prepared.pop(next(iter(prepared)))
        prepared[plan.key] = plan

    def coors_ready(self, coors: torch.Tensor) -> None:
        """Called by the detector as soon as the voxel coordinates are queued, before the perturber: the
        rulebooks (which depend on the coordinates only) are then built on a side stream concurrently
        with the perturber and the first GEMMs instead of after them."""
        if coors.is_cuda:
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(coors.device))
            self._coors_ready = (coors.data_ptr(), ev)

    FIN_SLOT = 1024   # ticket counters per fused BatchNorm finalize (rows up to 1023 * 32 * 64)

    def fin_tickets(self, device):
        """Zeroed ticket counters of the BatchNorm finalizes fused into the bf16 GEMMs (rpc_spconv_gemm_bf16_fin):
        one slot of FIN_SLOT counters per layer and direction (forward: slot li, backward: len(specs) + li);
        every launch leaves its counters zero again."""
        key = str(device)
        t = self.__dict__.setdefault("_fin_tickets", {}).get(key)
        if t is None:
            t = self._fin_tickets[key] = torch.zeros(2 * len(self.specs) * self.FIN_SLOT, dtype=torch.int32,
                                                     device=device)
        return t

    def fin_ticket_ptr(self, device, slot, n_rows):
        """Address of the ticket slot for a fused finalize over n_rows rows, or None (a separate finalize)
        when the rows need more counters than a slot holds."""
        lib = _ffi.load()
        if lib.rpc_bn_fin_tickets(max(int(n_rows), 1)) > self.FIN_SLOT:
            return None
        t = self.fin_tickets(device)
        return t.data_ptr() + 4 * slot * self.FIN_SLOT

    def grid(self, lvl, B, device):
        """Dense int32 index grid [B, D, H, W] kept all -1 between uses."""
        key = (lvl, B, str(device))
        g = self._grids.get(key)
        if g is None:
            D, H, W = self.shapes[lvl]
            g = torch.full((B * D * H * W,), -1, dtype=torch.int32, device=device)
            self._grids[key] = g
        return g

    def forward(self, voxel_features, coors, batch_size):
        params = []
        for m in self.layers():
            params += [m[0].weight, m[1].weight, m[1].bias]
        return SparseEncoderFn.apply(voxel_features, coors, self, int(batch_size), *params)


def _cdiv(a, b):
    return (a + b - 1) // b


def _r8(c):
    return (c + 7) // 8 * 8


def _r16(c):
    return (c + 15) // 16 * 16


def _r32(c):
    return (c + 31) // 32 * 32


def _prep_bf16_weights(lib, specs, Ws, dev, st, fwd_fmt=0):
    """Forward (format fwd_fmt: 0 bf16, 1 fp16) and data-gradient (bf16) B^T tiles of every 16-bit layer
    (entries of `specs` / `Ws`), from the fp32 master weights in rpc_spconv_prep_weight_bf16_batch launches of
    up to 32 tiles."""
    jobs = []
    for sp, W in zip(specs, Ws):
        for dg in (0, 1):
            bt = torch.empty(lib.rpc_spconv_bf16_weight_elems(sp.K, sp.ci, sp.co, dg), dtype=torch.bfloat16,
                             device=dev)
            jobs.append((sp, W, dg, bt))
    for g0 in range(0, len(jobs), 32):
        group = jobs[g0:g0 + 32]
        descs = (_ffi.RpcSpconvWprep * len(group))()
        for i, (sp, W, dg, bt) in enumerate(group):
            descs[i] = _ffi.RpcSpconvWprep(W.data_ptr(), bt.data_ptr(), sp.K, sp.ci, sp.co, dg,
                                           0 if dg else int(fwd_fmt))
        _ffi.check(lib.rpc_spconv_prep_weight_bf16_batch(descs, len(group), st), "rpc_spconv_prep_weight_bf16_batch")
    return [(jobs[2 * i][3], jobs[2 * i + 1][3]) for i in range(len(specs))]


def _bf16_dgrad_operands(lib, rec, dy, bnb, dev, st):
    """bf16 dz rows (BatchNorm backward applied) and the dgrad weight tiles W[k] (as B^T)."""
    sp = rec["spec"]
    dzb = torch.empty((rec["n_out"], _r8(sp.co)), dtype=torch.bfloat16, device=dev)
    _ffi.check(lib.rpc_bnbwd_to_bf16_rows(_ffi.ptr(dy), _ffi.ptr(rec["z"]), _ffi.ptr(bnb), rec["n_out"], sp.co,
                                          _ffi.ptr(dzb), st), "rpc_bnbwd_to_bf16_rows")
    btd = rec.get("btd")
    if btd is None:
        btd = torch.empty(lib.rpc_spconv_bf16_weight_elems(sp.K, sp.ci, sp.co, 1), dtype=torch.bfloat16, device=dev)
        _ffi.check(lib.rpc_spconv_prep_weight_bf16(_ffi.ptr(rec["W"]), sp.K, sp.ci, sp.co, 1, _ffi.ptr(btd), st),
                   "rpc_spconv_prep_weight_bf16")
    return dzb, btd


def _sparse_bytes(L, bf16, dense_bytes, backward):
    """Compulsory HBM bytes of the sparse encoder (stage_timer.py): per layer the input rows it gathers
    (bf16 rows in perf mode for layers >= 1), its rulebook and its output rows; backward adds the dz rows,
    the saved z and the data gradient; plus the dense BEV image (or its gradient) once."""
    total = dense_bytes
    for li, rec in enumerate(L):
        sp = rec["spec"]
        ein = 2 if (bf16 and li > 0) else 4
        n_in, n_out = rec["n_in"], rec["n_out"]
        fwd = n_in * sp.ci * ein + n_out * sp.K * 4 + n_out * sp.co * 4
        if not backward:
            total += fwd
        else:
            total += n_out * sp.co * 4 * 2 + n_out * sp.K * 4 + n_in * sp.ci * ein + n_in * sp.ci * 4
    return total


class KernelTimer:
    """HIP-event timing of sparse conv launches on the stream they are launched on.

    select: (op, ci, co) with op in {'fwd', 'dgrad', 'wgrad'}, or op None for every launch of every layer
    (bench.py's all-kernel roofline). Records per launch the event pair and the algorithmic FLOPs
    2 * pairs * ci * co (pairs = valid rulebook entries, counted on the device, read once at the end)."""

    def __init__(self, op=None, ci=None, co=None):
        self.sel = (op, ci, co)
        self.recs = []
        self.enabled = False
        self.kernel, self.dtype = None, None

    def wants(self, op, sp):
        return self.enabled and (self.sel[0] is None or self.sel == (op, sp.ci, sp.co))

    def reset(self):
        self.recs = []

    def start(self):
        e = torch.cuda.Event(enable_timing=True)
        e.record(torch.cuda.current_stream())
        return e

    def stop(self, e0, nbr, ci, co, kernel=None, dtype="fp32"):
        e1 = torch.cuda.Event(enable_timing=True)
        e1.record(torch.cuda.current_stream())
        self.recs.append((e0, e1, nbr, ci, co, kernel, dtype))   # pairs counted after the timed region
        self.kernel, self.dtype = kernel, dtype

    @staticmethod
    def _entry(recs):
        ms = sum(a.elapsed_time(b) for a, b, *_ in recs)
        flops = sum(2.0 * float((nbr >= 0).sum().item()) * ci * co for _, _, nbr, ci, co, _, _ in recs)
        n = len(recs)
        return dict(launches=n, avg_ms=ms / n, total_ms=ms, flops_per_launch=flops / n,
                    tflops=flops / (ms * 1e-3) / 1e12, kernel=recs[-1][5], dtype=recs[-1][6])

    def summary(self):
        """the selected launches as one entry (None if nothing was recorded)"""
        torch.cuda.synchronize()
        return self._entry(self.recs) if self.recs else None

    def per_kernel(self):
        """{kernel name: entry} over every recorded launch, grouped by kernel instantiation"""
        torch.cuda.synchronize()
        by = {}
        for r in self.recs:
            by.setdefault(r[5], []).append(r)
        return {k: self._entry(v) for k, v in by.items()}


class _RulebookPlan:
    """Every layer's rulebook on the encoder's 'rb' side stream: the submanifold neighbour lists (one
    per indice key) and, per strided conv, its output count, output coordinates and both neighbour maps.
    The chain depends on the coordinates only, so it starts from the detector's coors_ready event —
    concurrently with the perturber — and the main stream waits for each layer's event right before
    that layer's GEMM. Issued lazily, one level ahead: a strided conv's output count (a host read: it
    sizes the allocations) is read only when the forward reaches that layer, after the host has queued
    the previous level's GEMMs, so the main stream computes while the host waits."""

    def __init__(self, lib, enc, coors, n0, B, dev, after=None, consumer=None):
        """after: an event the coordinates are complete behind (default: the detector's coors_ready event,
        else everything queued on the current stream); consumer: the stream the GEMMs run on (default:
        the current stream)."""
        self.lib, self.enc, self.B, self.dev = lib, enc, B, dev
        self.main = consumer if consumer is not None else torch.cuda.current_stream(dev)
        self.side = enc.side_stream("rb", dev)
        self.key = (coors.data_ptr(), int(n0), int(B))
        self.coors0 = coors     # held: while this plan exists no other tensor can own that address
        ready = enc.__dict__.pop("_coors_ready", None)
        if after is not None:
            self.side.wait_event(after)
        elif ready is not None and ready[0] == coors.data_ptr():
            self.side.wait_event(ready[1])
        else:
            self.side.wait_stream(torch.cuda.current_stream(dev))
        coors.record_stream(self.side)
        self.plan = [None] * len(enc.specs)
        self.rb = {}
        self.pending = None        # (layer, n_host, event, ws, gout) of the issued strided count
        self.cur = (coors, n0)
        self.next = 0              # first layer not yet issued
        self._issue()

    def _done(self, li, p, made):
        ev = torch.cuda.Event()
        ev.record(self.side)
        p["ev"] = ev
        self.plan[li] = p
        for t in made:     # made on the side stream, used and freed on the main one
            t.record_stream(self.main)

    def _issue(self):
        """Issue layers from self.next up to (not including) the next strided conv, then its count."""
        lib, enc, dev, B = self.lib, self.enc, self.dev, self.B
        with torch.cuda.stream(self.side):
            st = _ffi.stream_of(self.cur[0])
            while self.next < len(enc.specs):
                li, sp = self.next, enc.specs[self.next]
                cur_coors, cur_n = self.cur
                if sp.kind != "subm":
                    oshp = _ffi.int_arr((B,) + enc.shapes[sp.lvl_out])
                    wsb = lib.rpc_spconv_rulebook_workspace_size(cur_n, sp.K)
                    ws = _ffi.workspace(wsb, dev)
                    n_dev = torch.empty(1, dtype=torch.int32, device=dev)
                    gout = enc.grid(sp.lvl_out, B, dev)
                    _ffi.check(lib.rpc_spconv_rulebook_count(_ffi.ptr(cur_coors), cur_n, oshp, _ffi.int_arr(sp.ksize),
                                                             _ffi.int_arr(sp.stride), _ffi.int_arr(sp.pad),
                                                             _ffi.ptr(gout), _ffi.ptr(n_dev), _ffi.ptr(ws), wsb, st),
                               "rpc_spconv_rulebook_count")
                    n_host = torch.empty(1, dtype=torch.int32, pin_memory=True)
                    n_host.copy_(n_dev, non_blocking=True)
                    ev = torch.cuda.Event()
                    ev.record(self.side)
                    self.pending = (li, n_host, ev, ws, gout)
                    return
                made = []
                if sp.key not in self.rb:
                    nbr = torch.empty((cur_n, sp.K), dtype=torch.int32, device=dev)
                    shp = _ffi.int_arr((B,) + enc.shapes[sp.lvl_in])
                    _ffi.check(lib.rpc_subm_rulebook(_ffi.ptr(cur_coors), cur_n, shp, _ffi.int_arr(sp.ksize),
                                                     _ffi.ptr(enc.grid(sp.lvl_in, B, dev)), _ffi.ptr(nbr), st),
                               "rpc_subm_rulebook")
                    self.rb[sp.key] = nbr
                    made.append(nbr)
                nbr = self.rb[sp.key]
                self._done(li, dict(n_in=cur_n, coors_in=cur_coors, nbr=nbr, n_out=cur_n, coors_out=cur_coors), made)
                self.next += 1

    def get(self, li):
        if self.plan[li] is None:
            lj, n_host, ev, ws, gout = self.pending
            assert lj == li, (lj, li)
            lib, enc, dev, B = self.lib, self.enc, self.dev, self.B
            sp = enc.specs[li]
            cur_coors, cur_n = self.cur
            ev.synchronize()
            n_out = int(n_host[0])             # host read: the strided conv's output row count
            with torch.cuda.stream(self.side):
                st = _ffi.stream_of(cur_coors)
                coors_out = torch.empty((n_out, 4), dtype=torch.int32, device=dev)
                nbr_out = torch.empty((n_out, sp.K), dtype=torch.int32, device=dev)
                nbr_in = torch.empty((cur_n, sp.K), dtype=torch.int32, device=dev)
                _ffi.check(lib.rpc_spconv_rulebook_build(_ffi.ptr(cur_coors), cur_n,
                                                         _ffi.int_arr((B,) + enc.shapes[sp.lvl_out]),
                                                         _ffi.int_arr(sp.ksize), _ffi.int_arr(sp.stride),
                                                         _ffi.int_arr(sp.pad), _ffi.ptr(gout), n_out,
                                                         _ffi.ptr(coors_out), _ffi.ptr(nbr_out), _ffi.ptr(nbr_in),
                                                         _ffi.ptr(ws), st), "rpc_spconv_rulebook_build")
            self._done(li, dict(n_in=cur_n, coors_in=cur_coors, nbr=nbr_out, nbr_in=nbr_in, n_out=n_out,
                                coors_out=coors_out), [coors_out, nbr_out, nbr_in])
            self.pending = None
            self.cur = (coors_out, n_out)
            self.next = li + 1
            self._issue()
        return self.plan[li]


class SparseEncoderFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, feats, coors, enc: SparseEncoder, B: int, *params):
        lib = _ffi.load()
        dev = feats.device
        st = _ffi.stream_of(feats)
        tm_stage = stage_timer.active()
        e_stage = stage_timer.TIMER.start() if tm_stage else None
        feats = feats.contiguous().float()
        coors = coors.to(torch.int32).contiguous()
        mods = enc.layers()
        src, src_bn = feats, None
        # perf mode: layers >= 1 gather bf16 rows of relu(bn(z)) (O(1) values); layer 0 stays fp32 —
        # its input is the raw VFE mean (coordinates up to 70 m, where a bf16 step is 0.5 m)
        bf16 = enc.bf16
        fmt = FWD_FMT if bf16 else 0     # forward operand format of the 16-bit layers
        hsrc = hwg = None
        L = []
        # 16-bit layers (1..): forward + data-gradient weight tiles of all of them in one launch
        wtiles = {}
        if bf16 and len(enc.specs) > 1:
            bl = list(range(1, len(enc.specs)))
            Ws = [params[3 * li].detach().float().contiguous() for li in bl]
            for li, tiles in zip(bl, _prep_bf16_weights(lib, [enc.specs[li] for li in bl], Ws, dev, st, fmt)):
                wtiles[li] = tiles
        # rulebooks (and the strided layers' output counts, host reads) on a side stream, ahead of the GEMMs
        plan = enc.__dict__.get("_prepared", {}).pop((coors.data_ptr(), feats.shape[0], B), None)
        if plan is None or plan.main != torch.cuda.current_stream(dev):
            plan = _RulebookPlan(lib, enc, coors, feats.shape[0], B, dev)
        else:
            enc.__dict__.pop("_coors_ready", None)
        main = torch.cuda.current_stream(dev)
        for li, (sp, m) in enumerate(zip(enc.specs, mods)):
            W = params[3 * li]
            gamma, beta = params[3 * li + 1], params[3 * li + 2]
            bnm = m[1]
            p = plan.get(li)
            rec = dict(spec=sp, n_in=p["n_in"], src=src, src_bn=src_bn, coors_in=p["coors_in"], nbr=p["nbr"],
                       n_out=p["n_out"], coors_out=p["coors_out"])
            if "nbr_in" in p:
                rec["nbr_in"] = p["nbr_in"]
            main.wait_event(p["ev"])
            n_out = rec["n_out"]
            z = torch.empty((n_out, sp.co), dtype=torch.float32, device=dev)
            nblk = max(lib.rpc_spconv_gemm_blocks(n_out), 1)
            part = torch.empty((nblk, 2 * sp.co), dtype=torch.float32, device=dev)
            tm = enc.timer is not None and enc.timer.wants("fwd", sp)
            rec["bf16"] = bf16 and li > 0
            rec["h_in"] = hwg if rec["bf16"] else None   # the weight gradient's bf16 rows
            rec["h_fmt"] = 0
            bn = torch.empty(4 * sp.co, dtype=torch.float32, device=dev)
            if rec["bf16"]:
                bt, rec["btd"] = wtiles[li]
                e0 = enc.timer.start() if tm else None
                _ffi.check(lib.rpc_spconv_gemm_h16(_ffi.ptr(hsrc), fmt, hsrc.shape[0], sp.ci, _ffi.ptr(rec["nbr"]),
                                                   sp.K, 0, n_out, _ffi.ptr(bt), sp.co, _ffi.ptr(z), None, None,
                                                   _ffi.ptr(part), 0, st), "rpc_spconv_gemm_h16")
            else:
                e0 = enc.timer.start() if tm else None
                _ffi.check(lib.rpc_spconv_forward(_ffi.ptr(src), _ffi.ptr(src_bn), sp.ci, _ffi.ptr(rec["nbr"]), sp.K,
                                                  n_out, _ffi.ptr(W), sp.co, _ffi.ptr(z), _ffi.ptr(part), st),
                           "rpc_spconv_forward")
            if tm:
                kn = (f"rpc::spb::k_gemm_bf16<{_r32(sp.ci)}, {_r16(sp.co) // 16}, 0>" if rec["bf16"] else
                      f"rpc::sp::k_gemm<{sp.ci}, {sp.co}, {1 if li else 0}, 0>")
                enc.timer.stop(e0, rec["nbr"], sp.ci, sp.co, kn, "bf16" if rec["bf16"] else "fp32")
            _ffi.check(lib.rpc_bn_finalize(_ffi.ptr(part), nblk, sp.co, n_out, 0, _ffi.ptr(gamma), _ffi.ptr(beta),
                                           float(bnm.eps), float(bnm.momentum), _ffi.ptr(bnm.running_mean),
                                           _ffi.ptr(bnm.running_var), None, _ffi.ptr(bn), None, None,
                                           None, st), "rpc_bn_finalize")
            rec.update(z=z, bn=bn, W=W, gamma=gamma, beta=beta)
            L.append(rec)
            if sp.mat:
                # materialised output rows: relu(bn(z) [+ block identity]) (+ the bf16 rows the next
                # layer gathers in perf mode)
                out = torch.empty((n_out, sp.co), dtype=torch.float32, device=dev)
                ob = (torch.empty((n_out, _r8(sp.co)), dtype=torch.bfloat16, device=dev)
                      if bf16 and li + 1 < len(enc.specs) else None)
                ob2 = torch.empty_like(ob) if ob is not None and fmt else None
                res = L[sp.res]["out"] if sp.res >= 0 else None
                _ffi.check(lib.rpc_sparse_res_forward_h16(_ffi.ptr(z), _ffi.ptr(bn), _ffi.ptr(res), n_out, sp.co,
                                                          _ffi.ptr(out), _ffi.ptr(ob), fmt, _ffi.ptr(ob2), st),
                           "rpc_sparse_res_forward_h16")
                rec["out"] = out
                src, src_bn, hsrc, hwg = out, None, ob, (ob2 if ob2 is not None else ob)
            else:
                src, src_bn = z, bn
                if bf16 and li + 1 < len(enc.specs):
                    # the next layer's gathered rows in the forward format, and (fp16 forward) a bf16 copy for its
                    # weight gradient, whose MFMAs pair them with the bf16 dz rows (one pass writes both: converting
                    # while the weight gradient stages them cost it 10 %)
                    hsrc = torch.empty((n_out, _r8(sp.co)), dtype=torch.bfloat16, device=dev)
                    hwg = torch.empty_like(hsrc) if fmt else hsrc
                    _ffi.check(lib.rpc_to_h16_rows(_ffi.ptr(z), _ffi.ptr(bn), n_out, sp.co, 1, fmt, _ffi.ptr(hsrc),
                                                   _ffi.ptr(hwg) if fmt else None, st), "rpc_to_h16_rows")
        _ffi.bump_batches([m[1] for m in mods])
        last = L[-1]
        D, H, Wd = enc.shapes[-1]
        C = last["spec"].co
        flags = (1 if enc.dense_nhwc else 0) | (2 if enc.dense_bf16 else 0)
        dt = torch.bfloat16 if enc.dense_bf16 else torch.float32
        # the dense BEV lives in one persistent buffer per module (re-zeroed each step): the SECOND
        # forward graph (dense_bev._graph_run) then reads it in place instead of from a copy
        # one buffer per shape: a returning shape (full batches after a partial last one) reuses the
        # storage its graph captured, and a dropped encoder frees them all
        # (at most the two most recent shapes are kept — e.g. full batches and a partial last one, or the
        # two engines' dtypes; a captured graph that still holds an evicted buffer keeps it alive itself and
        # copies from the new one when its shape returns)
        # Cleared where the previous step scattered (rpc_sparse_dense_clear on the coordinates it kept) rather
        # than zero-filled whole: 6 x 256 x 200 x 176 bf16 = 108 MB per step for SECOND against the ~10^4
        # occupied cells' bytes.
        bkey = (B, H, Wd, C * D, dt, enc.dense_nhwc, dev)
        bufs = enc.__dict__.setdefault("_dense_bufs", {})
        ent = bufs.pop(bkey, None)
        shp = _ffi.int_arr((B, D, H, Wd))
        if ent is None:
            while len(bufs) >= 2:
                bufs.pop(next(iter(bufs)))
            base = torch.empty((B, H, Wd, C * D) if enc.dense_nhwc else (B, C * D, H, Wd), dtype=dt, device=dev)
            dense_bev.mark_stable(base)
            base.zero_()
        else:
            base, prev_coors, prev_n = ent
            _ffi.check(lib.rpc_sparse_dense_clear(_ffi.ptr(prev_coors), prev_n, C, shp, flags, _ffi.ptr(base), st),
                       "rpc_sparse_dense_clear")
            # (the coordinates may come from a rulebook side stream: not reusable before this clear has run)
            prev_coors.record_stream(torch.cuda.current_stream(dev))
        # the coordinates kept for the next clear must be this step's own: a submanifold last layer's output
        # coordinates are its input's (possibly the caller's tensor, which it may refill in place) — keep a copy
        keep = last["coors_out"].clone() if last["spec"].kind == "subm" else last["coors_out"]
        bufs[bkey] = (base, keep, last["n_out"])      # most recently used last
        if enc.dense_nhwc:   # channels_last image, logically [B, C*D, H, W]
            dense = base.permute(0, 3, 1, 2)
        else:
            dense = base.view(base.shape)
        _ffi.check(lib.rpc_sparse_to_dense(_ffi.ptr(last["z"]), _ffi.ptr(last["bn"]), _ffi.ptr(last["coors_out"]),
                                           last["n_out"], C, shp, flags, _ffi.ptr(dense), st), "rpc_sparse_to_dense")
        if enc.flop_probe is not None:
            enc.flop_probe.append([(rec["nbr"], rec["spec"].ci, rec["spec"].co) for rec in L])
        if tm_stage:
            stage_timer.TIMER.stop("sparse_fwd", e_stage, _sparse_bytes(L, bf16, dense.numel() * dense.element_size(),
                                                                          backward=False))
        ctx.dense_flags = flags
        ctx.L = L
        ctx.enc = enc
        ctx.bf16 = bf16
        ctx.B = B
        ctx.shape = (B, C, D, H, Wd)
        ctx.n_feat = feats.shape
        return dense

    @staticmethod
    def backward(ctx, gdense):
        enc = ctx.enc
        timed = enc.timer is not None and enc.timer.enabled
        if NATIVE_BACKWARD and enc.debug is None and not timed:
            return _native_backward(ctx, gdense)
        lib = _ffi.load()
        L = ctx.L
        dev = gdense.device
        st = _ffi.stream_of(gdense)
        tm_stage = stage_timer.active()
        e_stage = stage_timer.TIMER.start() if tm_stage else None
        nbytes = _sparse_bytes(L, ctx.bf16, gdense.numel() * (2 if ctx.dense_flags & 2 else 4), backward=True) \
            if tm_stage else 0
        B, C, D, H, Wd = ctx.shape
        flags = ctx.dense_flags
        dt = torch.bfloat16 if flags & 2 else torch.float32
        if flags & 1:
            gd = gdense.to(dt).contiguous(memory_format=torch.channels_last)
        else:
            gd = gdense.to(dt).contiguous()
        grads = [None] * (3 * len(L))
        last = L[-1]
        n = last["n_out"]
        dy = torch.empty((n, C), dtype=torch.float32, device=dev)
        nblk = max(lib.rpc_spconv_gemm_blocks(n), 1)
        part = torch.empty((nblk, 2 * C), dtype=torch.float32, device=dev)
        _ffi.check(lib.rpc_dense_to_sparse_grad(_ffi.ptr(gd), _ffi.ptr(last["z"]), _ffi.ptr(last["bn"]),
                                                _ffi.ptr(last["coors_out"]), n, C, _ffi.int_arr((B, D, H, Wd)),
                                                flags, _ffi.ptr(dy), _ffi.ptr(part), st), "rpc_dense_to_sparse_grad")
        dfeat = None
        main = torch.cuda.current_stream(dev)
        wg = ctx.enc.side_stream("wg", dev)
        G = [[] for _ in L]     # gradient contributions to materialised outputs
        for li in range(len(L) - 1, -1, -1):
            rec = L[li]
            sp = rec["spec"]
            n_out = rec["n_out"]
            if sp.mat:
                # d out -> ReLU mask -> d(bn output); the block identity receives the same gradient
                g = G[li]
                nblk = max(lib.rpc_spconv_gemm_blocks(n_out), 1)
                if rec.get("res_m") is not None:   # done by the layer above's data-gradient epilogue
                    dy, part = rec.pop("res_m"), rec.pop("res_part")
                else:
                    dy = torch.empty((n_out, sp.co), dtype=torch.float32, device=dev)
                    part = torch.empty((nblk, 2 * sp.co), dtype=torch.float32, device=dev)
                    _ffi.check(lib.rpc_sparse_res_backward(_ffi.ptr(g[0]), _ffi.ptr(g[1] if len(g) > 1 else None),
                                                           _ffi.ptr(rec["out"]), _ffi.ptr(rec["z"]),
                                                           _ffi.ptr(rec["bn"]), n_out, sp.co, _ffi.ptr(dy),
                                                           _ffi.ptr(part), st), "rpc_sparse_res_backward")
                G[li] = None
                if sp.res >= 0:
                    G[sp.res].append(dy)
            if ctx.enc.debug is not None:
                ctx.enc.debug.append((li, rec["coors_out"].cpu().numpy(), rec["z"].detach().cpu().double(),
                                      dy.detach().cpu().double(), rec["bn"].detach().cpu().double(),
                                      rec["out"].detach().cpu() if rec.get("out") is not None else None))
            # BatchNorm backward statistics of this layer -> bnb, dgamma, dbeta
            bnb = torch.empty(5 * sp.co, dtype=torch.float32, device=dev)
            dgamma = torch.empty_like(rec["gamma"])
            dbeta = torch.empty_like(rec["beta"])
            _ffi.check(lib.rpc_bn_finalize(_ffi.ptr(part), nblk, sp.co, n_out, 1, _ffi.ptr(rec["gamma"]),
                                           _ffi.ptr(rec["beta"]), 0.0, 0.0, None, None, _ffi.ptr(rec["bn"]),
                                           _ffi.ptr(bnb), _ffi.ptr(dgamma), _ffi.ptr(dbeta), None, st),
                       "rpc_bn_finalize(bwd)")
            # weight gradient, on the 'wg' side stream: it reads only this layer's dz / input rows, so it
            # runs concurrently with the data-gradient chain of the main stream (both are gather-latency
            # bound with partial occupancy); the main stream joins it at the end of the backward
            dW = torch.empty_like(rec["W"])
            timer = ctx.enc.timer
            tw = timer is not None and timer.wants("wgrad", sp)
            dzb = btd = None
            if rec["bf16"]:
                dzb, btd = _bf16_dgrad_operands(lib, rec, dy, bnb, dev, st)
                ins = (rec["h_in"], rec["nbr"], dzb, dW)
            else:
                ins = (rec["src"], rec["src_bn"], rec["nbr"], dy, rec["z"], bnb, dW)
            ev = torch.cuda.Event()
            ev.record(main)
            wg.wait_event(ev)
            with torch.cuda.stream(wg):
                sw = _ffi.stream_of(dW)
                if rec["bf16"]:
                    wsz = lib.rpc_spconv_wgrad_bf16_workspace_size(n_out, sp.K, sp.ci, sp.co)
                    ws = _ffi.workspace(wsz, dev)
                    e0 = timer.start() if tw else None
                    _ffi.check(lib.rpc_spconv_wgrad_h16(_ffi.ptr(rec["h_in"]), rec["h_fmt"], sp.ci, _ffi.ptr(rec["nbr"]),
                                                        sp.K, n_out, _ffi.ptr(dzb), sp.co, _ffi.ptr(dW), _ffi.ptr(ws),
                                                        wsz, sw), "rpc_spconv_wgrad_h16")
                    kn = f"rpc::spb::k_wgrad_bf16<{sp.ci}, {sp.co}, 3>"
                else:
                    wsz = lib.rpc_spconv_wgrad_workspace_size(n_out, sp.K, sp.ci, sp.co)
                    ws = _ffi.workspace(wsz, dev)
                    e0 = timer.start() if tw else None
                    _ffi.check(lib.rpc_spconv_wgrad(_ffi.ptr(rec["src"]), _ffi.ptr(rec["src_bn"]), sp.ci,
                                                    _ffi.ptr(rec["nbr"]), sp.K, n_out, _ffi.ptr(dy), _ffi.ptr(rec["z"]),
                                                    _ffi.ptr(bnb), sp.co, _ffi.ptr(dW), _ffi.ptr(ws), wsz, sw),
                               "rpc_spconv_wgrad")
                    kn = f"rpc::sp::k_wgrad<{sp.ci}, {sp.co}, {1 if li else 0}>"
                if tw:
                    timer.stop(e0, rec["nbr"], sp.ci, sp.co, kn, "bf16" if rec["bf16"] else "fp32")
            for t in ins:
                if t is not None:
                    t.record_stream(wg)
            grads[3 * li: 3 * li + 3] = [dW, dgamma, dbeta]
            # data gradient into the previous layer (ReLU mask + its BN-backward partial sums)
            n_in = rec["n_in"]
            if sp.kind == "subm":
                mp, rev = rec["nbr"], 1
            else:
                mp, rev = rec["nbr_in"], 0
            din = torch.empty((n_in, sp.ci), dtype=torch.float32, device=dev)
            td = timer is not None and timer.wants("dgrad", sp) and (li > 0 or ctx.needs_input_grad[0])
            e0 = timer.start() if td else None
            epi = 2    # the data-gradient epilogue: 1 = BN-backward partial rows, 2 = plain, 3 = residual (E_RES)
            if li > 0 and L[li - 1]["spec"].mat and rec["bf16"] and lib.rpc_sparse_tune(0, -1) and len(G[li - 1]) <= 1:
                epi = 3
                # the input is a block output: its residual backward in this data gradient's epilogue
                # (rpc_spconv_gemm_res), as rpc_sparse_backward does
                prev = L[li - 1]
                nb = max(lib.rpc_spconv_gemm_blocks(n_in), 1)
                pp = torch.empty((nb, 2 * sp.ci), dtype=torch.float32, device=dev)
                gid = G[li - 1][0] if G[li - 1] else None
                _ffi.check(lib.rpc_spconv_gemm_res(_ffi.ptr(dzb), dzb.shape[0], sp.co, _ffi.ptr(mp), sp.K, rev,
                                                   n_in, _ffi.ptr(btd), sp.ci, _ffi.ptr(din),
                                                   _ffi.ptr(gid), _ffi.ptr(prev["out"]), _ffi.ptr(prev["z"]),
                                                   _ffi.ptr(prev["bn"]), _ffi.ptr(pp), None, st), "rpc_spconv_gemm_res")
                prev["res_m"], prev["res_part"] = din, pp
            elif li > 0 and L[li - 1]["spec"].mat:
                # the input is a materialised output: plain data gradient, masked by its own backward
                if rec["bf16"]:
                    _ffi.check(lib.rpc_spconv_gemm_h16(_ffi.ptr(dzb), 0, dzb.shape[0], sp.co, _ffi.ptr(mp), sp.K, rev, n_in,
                                                        _ffi.ptr(btd), sp.ci, _ffi.ptr(din), None, None, None, 2, st),
                               "rpc_spconv_gemm_h16(dgrad)")
                else:
                    _ffi.check(lib.rpc_spconv_dgrad(_ffi.ptr(dy), _ffi.ptr(rec["z"]), _ffi.ptr(bnb), sp.co,
                                                    _ffi.ptr(mp), sp.K, rev, n_in, _ffi.ptr(rec["W"]), sp.ci, None,
                                                    None, _ffi.ptr(din), None, st), "rpc_spconv_dgrad")
                G[li - 1].append(din)
            elif li > 0:
                prev = L[li - 1]
                nblk = max(lib.rpc_spconv_gemm_blocks(n_in), 1)
                part = torch.empty((nblk, 2 * sp.ci), dtype=torch.float32, device=dev)
                epi = 1
                if rec["bf16"]:
                    _ffi.check(lib.rpc_spconv_gemm_h16(_ffi.ptr(dzb), 0, dzb.shape[0], sp.co, _ffi.ptr(mp), sp.K, rev, n_in,
                                                        _ffi.ptr(btd), sp.ci, _ffi.ptr(din), _ffi.ptr(prev["z"]),
                                                        _ffi.ptr(prev["bn"]), _ffi.ptr(part), 1, st),
                               "rpc_spconv_gemm_h16(dgrad)")
                else:
                    _ffi.check(lib.rpc_spconv_dgrad(_ffi.ptr(dy), _ffi.ptr(rec["z"]), _ffi.ptr(bnb), sp.co,
                                                    _ffi.ptr(mp), sp.K, rev, n_in, _ffi.ptr(rec["W"]), sp.ci,
                                                    _ffi.ptr(prev["z"]), _ffi.ptr(prev["bn"]), _ffi.ptr(din),
                                                    _ffi.ptr(part), st), "rpc_spconv_dgrad")
                dy = din
            elif ctx.needs_input_grad[0]:
                if rec["bf16"]:
                    _ffi.check(lib.rpc_spconv_gemm_h16(_ffi.ptr(dzb), 0, dzb.shape[0], sp.co, _ffi.ptr(mp), sp.K, rev, n_in,
                                                        _ffi.ptr(btd), sp.ci, _ffi.ptr(din), None, None, None, 2, st),
                               "rpc_spconv_gemm_h16(dgrad)")
                else:
                    _ffi.check(lib.rpc_spconv_dgrad(_ffi.ptr(dy), _ffi.ptr(rec["z"]), _ffi.ptr(bnb), sp.co,
                                                    _ffi.ptr(mp), sp.K, rev, n_in, _ffi.ptr(rec["W"]), sp.ci, None,
                                                    None, _ffi.ptr(din), None, st), "rpc_spconv_dgrad")
                dfeat = din
            if td:
                kn = (f"rpc::spb::k_gemm_bf16<{_r32(sp.co)}, {_r16(sp.ci) // 16}, {epi}>" if rec["bf16"] else
                      f"rpc::sp::k_gemm<{sp.co}, {sp.ci}, 2, {1 if epi == 1 else 0}>")
                timer.stop(e0, rec["nbr"], sp.ci, sp.co, kn, "bf16" if rec["bf16"] else "fp32")
        main.wait_stream(wg)    # the weight gradients are complete before autograd hands them on
        if tm_stage:
            stage_timer.TIMER.stop("sparse_bwd", e_stage, nbytes)
        ctx.L = None
        ctx.enc = None
        return (dfeat, None, None, None, *grads)


def _native_backward(ctx, gdense):
    """SparseEncoderFn.backward as ONE C-ABI call (rpc_sparse_backward, csrc/sparse_exec.hip): the same
    kernels with the same arguments in the same order as the per-layer loop above, issued from C++
    (the loop's host time exceeded the GPU time of its kernels). Gradients of all layers land in one
    flat buffer (views returned to autograd)."""
    lib = _ffi.load()
    L = ctx.L
    dev = gdense.device
    main = torch.cuda.current_stream(dev)
    st = _ffi.stream_of(gdense)
    tm_stage = stage_timer.active()
    e_stage = stage_timer.TIMER.start() if tm_stage else None
    B, C, D, H, Wd = ctx.shape
    flags = ctx.dense_flags
    dt = torch.bfloat16 if flags & 2 else torch.float32
    gd = gdense.to(dt).contiguous(memory_format=torch.channels_last) if flags & 1 else gdense.to(dt).contiguous()
    nl = len(L)
    sizes = []
    for rec in L:
        sizes += [rec["W"].numel(), rec["gamma"].numel(), rec["beta"].numel()]
    flat = torch.empty(sum(sizes), dtype=torch.float32, device=dev)
    parts = torch.split(flat, sizes)
    grads = []
    table = (_ffi.RpcSparseLayer * nl)()
    vp = lambda t: None if t is None else t.data_ptr()
    for li, rec in enumerate(L):
        sp = rec["spec"]
        dW = parts[3 * li].view(rec["W"].shape)
        dg, db = parts[3 * li + 1], parts[3 * li + 2]
        grads += [dW, dg, db]
        bf = bool(rec["bf16"])
        if bf and rec.get("btd") is None:
            btd = torch.empty(lib.rpc_spconv_bf16_weight_elems(sp.K, sp.ci, sp.co, 1), dtype=torch.bfloat16, device=dev)
            _ffi.check(lib.rpc_spconv_prep_weight_bf16(_ffi.ptr(rec["W"]), sp.K, sp.ci, sp.co, 1, _ffi.ptr(btd), st),
                       "rpc_spconv_prep_weight_bf16")
            rec["btd"] = btd
        table[li] = _ffi.RpcSparseLayer(
            0 if sp.kind == "subm" else 1, sp.ci, sp.co, sp.K, rec["n_in"], rec["n_out"], int(bf), int(sp.mat),
            sp.res, vp(rec["nbr"]), vp(rec.get("nbr_in")), vp(rec["z"]), vp(rec["bn"]), vp(rec.get("out")),
            vp(rec["h_in"]) if bf else None, None if bf else vp(rec["src"]), None if bf else vp(rec["src_bn"]),
            vp(rec["W"]), vp(rec["gamma"]), vp(rec["beta"]), vp(rec.get("btd")) if bf else None,
            dW.data_ptr(), dg.data_ptr(), db.data_ptr(), int(rec.get("h_fmt", 0)),
            ctx.enc.fin_ticket_ptr(dev, nl + li, rec["n_in"]) if bf and FUSED_FINALIZE else None)
    dfeat = (torch.empty((L[0]["n_in"], L[0]["spec"].ci), dtype=torch.float32, device=dev)
             if ctx.needs_input_grad[0] else None)
    wsb = lib.rpc_sparse_backward_workspace_size(table, nl)
    if wsb == 0:
        raise RuntimeError("rpc_sparse_backward_workspace_size: inconsistent layer table")
    ws = _ffi.workspace(wsb, dev)
    wg = ctx.enc.side_stream("wg", dev)
    _ffi.check(lib.rpc_sparse_backward(table, nl, _ffi.ptr(gd), _ffi.ptr(L[-1]["coors_out"]),
                                       _ffi.int_arr((B, D, H, Wd)), flags, _ffi.ptr(dfeat), _ffi.ptr(ws), wsb, st,
                                       C_stream(wg)), "rpc_sparse_backward")
    if tm_stage:
        stage_timer.TIMER.stop("sparse_bwd", e_stage, _sparse_bytes(L, ctx.bf16, gdense.numel() * (2 if flags & 2 else 4),
                                                                      backward=True))
    ctx.L = None
    ctx.enc = None
    return (dfeat, None, None, None, *grads)


def C_stream(s):
    import ctypes
    return ctypes.c_void_p(s.cuda_stream)

