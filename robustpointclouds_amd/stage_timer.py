"""HIP-event timing of the HBM-bound stages of the step (SURVEY.md §8(d) per-stage roofline).

bench.py turns `TIMER.enabled` on for a few eager steps after its timed loop. Each stage records an
event pair on the stream it is launched on plus its COMPULSORY bytes — what the stage must read and
write at least once (inputs, outputs, index tables), not what the kernels actually move — so
bytes / time / 8 TB/s is the stage's fraction of the HBM roofline:

* voxelize (rpc_hard_voxelize):   P·F·4 points in + V·(T·F·4 + 16 + 4) voxels / coors / counts out
* perturber fwd (rpc_perturber_forward, fused a2/a3/a5): V·T·F·4 voxels + V·4 counts in,
  V·T·F·4 perturbed voxels + V·vf·4 VFE out
* perturber bwd: V·T·F·4 voxels + V·4 + V·vf·4 dVFE in (parameter gradients are ~0.1 MB)
* sparse fwd (12 convs): per layer the gathered input rows (n_in·C_in, bf16 or fp32), the rulebook
  (n_out·K·4), the output rows (n_out·C_out·4), plus the dense BEV image written once
* sparse bwd: per layer dz rows in (n_out·C_out·4), the rulebook, the saved z and input rows for the
  weight gradient, the data gradient out (n_in·C_in·4), plus the dense BEV gradient read once

Sizes that are device values at launch time (the voxel count V) are kept as device tensors and read
in `summary()`, after the timed region.
"""
from __future__ import annotations

from collections import defaultdict

import torch

HBM_PEAK_GBPS = 8000.0   # MI355X HBM3E, /opt/skills/guides/MI355X_MICROARCH.md


class StageTimer:
    def __init__(self):
        self.enabled = False
        self.recs = defaultdict(list)

    def start(self, stream=None):
        e = torch.cuda.Event(enable_timing=True)
        e.record(stream if stream is not None else torch.cuda.current_stream())
        return e

    def stop(self, stage, e0, nbytes, stream=None):
        """nbytes: an int, or a callable evaluated in summary() (for device-side sizes)."""
        e1 = torch.cuda.Event(enable_timing=True)
        e1.record(stream if stream is not None else torch.cuda.current_stream())
        self.recs[stage].append((e0, e1, nbytes))

    def reset(self):
        self.recs = defaultdict(list)

    def summary(self):
        torch.cuda.synchronize()
        out = {}
        for stage, rs in self.recs.items():
            ms = sum(a.elapsed_time(b) for a, b, _ in rs)
            byts = sum(float(n() if callable(n) else n) for _, _, n in rs)
            n = len(rs)
            gbps = byts / (ms * 1e-3) / 1e9 if ms > 0 else 0.0
            out[stage] = dict(launches=n, avg_ms=round(ms / n, 4), bytes_per_launch=round(byts / n),
                              achieved_gbps=round(gbps, 1), peak_gbps=HBM_PEAK_GBPS,
                              frac=round(gbps / HBM_PEAK_GBPS, 4))
        return out


TIMER = StageTimer()


def active() -> bool:
    return TIMER.enabled and not torch.cuda.is_current_stream_capturing()
