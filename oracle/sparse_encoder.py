"""PARITY ORACLE — TEST INFRASTRUCTURE ONLY.

CPU restatement of upstream mmdet3d `SparseEncoder` over spconv (spconv-cu113>=2.3.0,
requirements.txt:18; config adversarial-second_hv_secfpn_8xb6-80e_kitti-3d-3class.py:19-23;
call site models/detectors/adversarial_voxelnet.py:141). spconv/mmdet3d are not in this
container and the reference holds no vectors for this layer, so this
is "parity unpinned" w.r.t. spconv itself: it restates spconv's published semantics —
  SubMConv3d:   out(o) = sum_k W[k]^T in(o + k - centre), output sites = input sites
  SparseConv3d: out(o) = sum_k W[k]^T in(o*s - p + k), output sites = every o reached
                by an input; spatial out = (in + 2p - (k-1) - 1)//s + 1
  BatchNorm1d (train: batch stats, biased var; running stats with the unbiased var),
  ReLU, `.dense()` -> [B, C, D, H, W] -> view(B, C*D, H, W);
  SparseBasicBlock (block_type='basicblock'): relu(bn2(conv2(relu(bn1(conv1(x))))) + x)
with numpy index arithmetic and torch float64 autograd on CPU (gather / matmul /
index_add). Row ORDER of intermediate sparse tensors is free (the dense output and the
BatchNorm statistics do not depend on it).
"""
from __future__ import annotations

import numpy as np
import torch


def _keys(c, shape):
    B, D, H, W = shape
    c = c.astype(np.int64)
    return ((c[:, 0] * D + c[:, 1]) * H + c[:, 2]) * W + c[:, 3]


def subm_pairs(coors, shape, ksize=(3, 3, 3)):
    """list over k of (in_rows, out_rows)"""
    keys = _keys(coors, shape)
    order = np.argsort(keys)
    sk = keys[order]
    B, D, H, W = shape
    pairs = []
    kz, ky, kx = ksize
    for a in range(kz):
        for b in range(ky):
            for c in range(kx):
                off = np.array([0, a - kz // 2, b - ky // 2, c - kx // 2])
                nb = coors + off
                ok = (nb[:, 1] >= 0) & (nb[:, 1] < D) & (nb[:, 2] >= 0) & (nb[:, 2] < H) & (nb[:, 3] >= 0) & (nb[:, 3] < W)
                nk = _keys(nb, shape)
                pos = np.clip(np.searchsorted(sk, nk), 0, len(sk) - 1)
                hit = ok & (sk[pos] == nk) if len(sk) else ok & False
                out_rows = np.nonzero(hit)[0]
                in_rows = order[pos[hit]]
                pairs.append((in_rows, out_rows))
    return pairs


def spconv_pairs(coors, out_shape, ksize, stride, pad):
    """(out_coors, list over k of (in_rows, out_rows))"""
    B, D, H, W = out_shape
    cands = []
    kz, ky, kx = ksize
    ks = []
    for a in range(kz):
        for b in range(ky):
            for c in range(kx):
                n = coors[:, 1:] + np.array(pad) - np.array([a, b, c])
                ok = np.all(n >= 0, 1) & np.all(n % np.array(stride) == 0, 1)
                o = n // np.array(stride)
                ok &= (o[:, 0] < D) & (o[:, 1] < H) & (o[:, 2] < W)
                oc = np.concatenate([coors[:, :1], o], 1)
                ks.append((np.nonzero(ok)[0], oc[ok]))
    allc = np.concatenate([oc for _, oc in ks]) if ks else np.zeros((0, 4), np.int64)
    ukeys, first = np.unique(_keys(allc, out_shape), return_index=True)
    out_coors = allc[first]
    pairs = []
    for rows, oc in ks:
        o = np.searchsorted(ukeys, _keys(oc, out_shape))
        pairs.append((rows, o))
    return out_coors.astype(np.int64), pairs


def _bf16(t):
    return t.to(torch.bfloat16).to(t.dtype)


def _match(c_to, c_from, rows):
    """rows given in the order of coordinates c_from, reordered to the order of c_to (the same coordinate set)"""
    kf, kt = _keys(c_from, (1 << 8, 1 << 8, 1 << 12, 1 << 12)), _keys(c_to, (1 << 8, 1 << 8, 1 << 12, 1 << 12))
    order = np.argsort(kf)
    pos = order[np.searchsorted(kf, kt, sorter=order)]
    assert np.array_equal(kf[pos], kt)
    return rows[pos]


def _fp16(t):
    return t.to(torch.float16).to(t.dtype)


class _RoundFwd(torch.autograd.Function):
    """bf16 (or fp16) rounding of a GEMM operand in the forward; the gradient passes through unrounded."""

    @staticmethod
    def forward(ctx, x, fp16=False):
        return _fp16(x) if fp16 else _bf16(x)

    @staticmethod
    def backward(ctx, g):
        return g, None


class _RoundBwd(torch.autograd.Function):
    """Identity in the forward; the gradient arriving at a conv output (the BatchNorm-backward dz that the
    perf mode stores as bf16 rows before its data- and weight-gradient GEMMs) rounded to bf16."""

    @staticmethod
    def forward(ctx, x):
        return x.clone()

    @staticmethod
    def backward(ctx, g):
        return _bf16(g)


class OracleSparseEncoder:
    """SECOND SparseEncoder with explicit float64 weights copied from a GPU module.

    bf16_from (optional layer index): emulate the perf mode's 16-bit GEMM operands from that layer on — the
    gathered input rows relu(bn(z)) and the weights rounded to bf16 (fwd_fp16: to fp16) in the forward, the
    BatchNorm-backward dz rounded to bf16 before the data / weight gradients — with every other operation in
    `dtype`: the error an implementation with those operands cannot avoid (the bar of
    tests/test_gpu_sparse_layers.py)."""

    def __init__(self, enc, dtype=torch.float64, bf16_from=None, fwd_fp16=False):
        self.specs = enc.specs
        self.shapes = enc.shapes
        self.dtype = dtype
        self.bf16_from = bf16_from
        self.fwd_fp16 = fwd_fp16
        self.params = []
        for m in enc.layers():
            W = m[0].weight.detach().cpu().to(dtype).clone().requires_grad_(True)
            g = m[1].weight.detach().cpu().to(dtype).clone().requires_grad_(True)
            b = m[1].bias.detach().cpu().to(dtype).clone().requires_grad_(True)
            self.params.append(dict(W=W, g=g, b=b, eps=m[1].eps, mom=m[1].momentum,
                                    rm=m[1].running_mean.detach().cpu().to(dtype).clone(),
                                    rv=m[1].running_var.detach().cpu().to(dtype).clone()))

    def forward(self, feats, coors, B, keep=False, masks=None, flips=None):
        """masks (optional): per layer (coors, bool [n, co]) — the ReLU decisions of the implementation under test,
        rows matched here by coordinates; the layer's output is then (pre [+ identity]) * mask instead of relu(...):
        float64 arithmetic on the implementation's own branch of the piecewise-linear encoder. A pre-activation
        within an fp32 rounding of 0 lands on either side in fp32; evaluated on the other branch, one such element
        moved every gradient below its layer by ~1e-3 (tests/test_gpu_sparse_layers.py).
        flips (optional, with masks; tests/_dense_masks.FlipStats or any object with `flips`, `worst`, `per_layer`):
        every adopted decision that differs from this oracle's own (act > 0) is counted, and `worst` records the
        largest |act| / max |act| of its channel over them — how far from zero an adopted decision may lie is
        bounded by the tests (FLIP_PRE_MAX), so a wrong-sign kernel is not copied into the oracle unseen."""
        x = torch.as_tensor(feats).to(self.dtype)
        c = np.asarray(coors, np.int64)
        cache = {}
        self.trace = []   # keep=True: per layer (coors, z pre-BN, pre-activation) for debugging
        outs = []         # per layer output features (SparseBasicBlock identities)
        for li, (sp, p) in enumerate(zip(self.specs, self.params)):
            if sp.kind == "subm":
                if sp.key not in cache:
                    cache[sp.key] = subm_pairs(c, (B,) + self.shapes[sp.lvl_in], sp.ksize)
                pairs, n_out, c_out = cache[sp.key], x.shape[0], c
            else:
                c_out, pairs = spconv_pairs(c, (B,) + self.shapes[sp.lvl_out], sp.ksize, sp.stride, sp.pad)
                n_out = c_out.shape[0]
            q = self.bf16_from is not None and li >= self.bf16_from
            xg, Wg = (_RoundFwd.apply(x, self.fwd_fp16), _RoundFwd.apply(p["W"], self.fwd_fp16)) if q else (x, p["W"])
            z = torch.zeros((n_out, sp.co), dtype=self.dtype)
            for k, (ri, ro) in enumerate(pairs):
                if len(ri):
                    z = z.index_add(0, torch.from_numpy(ro), xg[torch.from_numpy(ri)] @ Wg[k])
            if q:
                z = _RoundBwd.apply(z)
            mean = z.mean(0)
            var = z.var(0, unbiased=False)
            with torch.no_grad():
                n = z.shape[0]
                p["rm"] = (1 - p["mom"]) * p["rm"] + p["mom"] * mean
                p["rv"] = (1 - p["mom"]) * p["rv"] + p["mom"] * var * n / max(n - 1, 1)
            pre = (z - mean) / torch.sqrt(var + p["eps"]) * p["g"] + p["b"]
            if keep:
                pre.retain_grad()
                self.trace.append((c_out, z, pre))
            res = getattr(sp, "res", -1)
            act = pre + outs[res] if res >= 0 else pre                         # SparseBasicBlock: + identity
            if masks is not None:
                mc, mm = masks[li]
                m = torch.from_numpy(_match(c_out, np.asarray(mc), np.asarray(mm)))
                if flips is not None:
                    a = act.detach()
                    d = m != (a > 0)
                    nd = int(d.sum())
                    w = 0.0
                    if nd:
                        sc = a.abs().amax(0, keepdim=True).clamp_min(1e-30)
                        w = float((a.abs() / sc)[d].max())
                        flips.flips += nd
                        flips.worst = max(flips.worst, w)
                    if hasattr(flips, "per_layer"):
                        flips.per_layer.append((li, nd, w))
                x = act * m.to(self.dtype)
            else:
                x = torch.relu(act)
            outs.append(x)
            c = c_out
        D, H, W = self.shapes[-1]
        C = x.shape[1]
        dense = torch.zeros((B, D, H, W, C), dtype=self.dtype)
        idx = (torch.from_numpy(c[:, 0]), torch.from_numpy(c[:, 1]), torch.from_numpy(c[:, 2]),
               torch.from_numpy(c[:, 3]))
        dense = dense.index_put(idx, x)
        return dense.permute(0, 4, 1, 2, 3).reshape(B, C * D, H, W)


def implementation_masks(debug):
    """The ReLU decisions of the HIP SparseEncoder from its debug trace (SparseEncoder.debug: per layer (layer,
    coors, z, dy, bn, out)), for OracleSparseEncoder.forward(masks=...): out > 0 for materialised layers (the
    kernel's own relu(bn(z) + identity)), else the kernels' fmaxf(fmaf(z - mean, scale, beta), 0) > 0 — z - mean
    rounded in fp32 as the kernel does, the fused multiply-add's sign that of its exact value (exact in float64)."""
    masks = []
    for li, c, z, dy, bn, out in sorted(debug, key=lambda t: t[0]):
        if out is not None:
            m = (out > 0).numpy()
        else:
            C = z.shape[1]
            a = (z.float() - bn[2 * C:3 * C].float()).double()
            m = (a * bn[:C].float().double() + bn[C:2 * C].float().double() > 0).numpy()
        masks.append((c, m))
    return masks

