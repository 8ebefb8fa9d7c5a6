"""Same-branch parity for the dense BEV stack (SECOND backbone + SECONDFPN neck): the float64 / fp32 torch
oracle evaluated on the HIP engine's ReLU decisions.

A Conv-BN-ReLU whose pre-activation sits within fp32 rounding of zero is decided differently by any two fp32
implementations (and by float64); one flipped decision at a pixel carrying a large gradient moves that layer's
BatchNorm-bias gradient (sum dm) and every gradient below it by ~1e-2 (tools/dbg_cp_bb.py, r05: HIP 1.3e-2 vs
fp32 torch 4e-4 at blocks.1.6 of the CenterPoint backbone, with dgamma of the same layer at 6e-5 — the flip
is at x_hat ~ 0). The oracle therefore multiplies each ReLU's input by the engine's decision (exactly the
kernel's: sign of fmaf(z - mean, scale, beta) on the stored fp32 values), and the tests bound separately how
far from zero every decision that differs from the oracle's own lies (`FlipStats.worst`: |pre| relative to
the channel's max |pre|)."""
import torch
from torch import nn


def engine_masks(trace):
    """dense_bev.DEBUG entries (bn module, z [Mo][co], bn [4co] = scale, beta, mean, invstd, B, Ho, Wo) ->
    {id(bn module): bool mask [B, co, Ho, Wo] on the CPU}. The fp32 difference z - mean is the kernel's; the
    product with scale is exact in double and the sum with beta keeps the sign of fmaf's exact result."""
    out = {}
    for bnm, z, bn, B, Ho, Wo in trace:
        co = z.shape[1]
        sc, be, mu = bn[:co], bn[co:2 * co], bn[2 * co:3 * co]
        pre = (z.float() - mu.float()).double() * sc.double() + be.double()
        out[id(bnm)] = (pre > 0).view(B, Ho, Wo, co).permute(0, 3, 1, 2).contiguous().cpu()
    return out


class FlipStats:
    """Adopted ReLU decisions that differ from the oracle's own: used by follow_masks (dense) and by
    oracle/sparse_encoder.OracleSparseEncoder.forward(flips=...) (sparse)."""

    def __init__(self):
        self.flips = 0
        self.worst = 0.0   # max |pre| / max_channel |pre| over the flipped decisions
        self.per_layer = []   # sparse: (layer, differing decisions, worst) per layer

    def __repr__(self):
        return f"FlipStats(flips={self.flips}, worst={self.worst:.3e})"


def follow_masks(hip_mods, ref_mods, masks, stats=None):
    """Install forward hooks on every ReLU of the oracle modules ref_mods (deep copies of hip_mods): the ReLU
    after the k-th BatchNorm2d passes its input times the engine's mask of the k-th BatchNorm2d of hip_mods.
    Returns the hook handles."""
    hip_bns = [m for hm in hip_mods for m in hm.modules() if isinstance(m, nn.BatchNorm2d)]
    handles = []
    k = 0
    for rm in ref_mods:
        for seq in rm.modules():
            if not isinstance(seq, nn.Sequential):
                continue
            kids = list(seq.children())
            for a, b in zip(kids, kids[1:]):
                if isinstance(a, nn.BatchNorm2d) and isinstance(b, nn.ReLU):
                    mask = masks[id(hip_bns[k])]
                    k += 1
                    b.inplace = False

                    def hook(mod, inp, out, mask=mask):
                        x = inp[0]
                        m = mask.to(device=x.device)
                        if stats is not None:
                            d = m != (x > 0)
                            if bool(d.any()):
                                sc = x.detach().abs().amax(dim=(0, 2, 3), keepdim=True).clamp_min(1e-30)
                                stats.flips += int(d.sum())
                                stats.worst = max(stats.worst, float((x.detach().abs() / sc)[d].max()))
                        return x * m.to(x.dtype)
                    handles.append(b.register_forward_hook(hook))
    assert k == len(hip_bns) == len(masks), (k, len(hip_bns), len(masks))
    return handles
