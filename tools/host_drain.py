"""Where the training stream runs dry inside a bench step: an event is recorded on the training stream at each
phase boundary of Trainer.train_step (entry, forward issued, backward issued, batch prefetch done, optimizer
issued, exit); when the host reaches a boundary it also asks whether the previous boundary's event has already
completed on the GPU. A completed event means every kernel issued before it had run: the stream was (or is about
to be) idle while the host worked on the phase in between. Prints per phase: GPU ms between the boundary events,
the fraction of steps whose stream had drained by the end of the phase's host work, and host ms of the phase.

    python tools/host_drain.py [--steps 30]
"""
import argparse
import collections
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from robustpointclouds_amd import trainer as T  # noqa: E402

REC = []     # per step: list of (name, event, drained_flag, host_t)


def mark(name):
    if not REC:
        return
    cur = REC[-1]
    drained = cur[-1][1].query() if cur else False
    e = torch.cuda.Event(enable_timing=True)
    e.record()
    cur.append((name, e, drained, time.perf_counter()))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=30)
    a = ap.parse_args()
    dev = torch.device("cuda")
    torch.manual_seed(0)
    model = T.make_kitti_model(num_classes=3, device=dev, epoch=3)
    tr = T.Trainer(model, bf16=True, device=dev)
    orig_up = T.Trainer.update_params

    def update_params(self, loss):
        mark("forward")
        loss.backward()
        mark("backward")
        self._issue_prefetch()
        mark("prefetch")
        if isinstance(self.opt, T.ClipAdamW):
            self._grad_norm = self.opt.step()[0]
        else:
            self._grad_norm = torch.nn.utils.clip_grad_norm_(self.module.parameters(), self.max_norm)
            self.opt.step()
        self.opt.zero_grad(set_to_none=True)
        mark("optimizer")
    T.Trainer.update_params = update_params
    data = bench._batches(4, 6, 0, dev, 3)
    ready = torch.cuda.Event()
    ready.record()
    for i in range(8):
        tr.train_step(*data[i % 4], next_points=data[(i + 1) % 4][0], next_ready=ready)
    torch.cuda.synchronize()
    for i in range(a.steps):
        REC.append([])
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        REC[-1].append(("start", e, False, time.perf_counter()))
        tr.train_step(*data[i % 4], next_points=data[(i + 1) % 4][0], next_ready=ready)
        mark("end")
    torch.cuda.synchronize()
    T.Trainer.update_params = orig_up
    gpu, host, dr = collections.defaultdict(list), collections.defaultdict(list), collections.defaultdict(int)
    for i, st in enumerate(REC):
        for (n0, e0, _, h0), (n1, e1, d1, h1) in zip(st, st[1:]):
            gpu[n1].append(e0.elapsed_time(e1))
            host[n1].append((h1 - h0) * 1e3)
            dr[n1] += int(d1)
        if i + 1 < len(REC):
            n = "next-step start"
            gpu[n].append(st[-1][1].elapsed_time(REC[i + 1][0][1]))
            host[n].append((REC[i + 1][0][3] - st[-1][3]) * 1e3)
    tot = REC[0][0][1].elapsed_time(REC[-1][-1][1]) / a.steps
    print(f"{a.steps} steps, {tot:.3f} ms/step (GPU, first start to last end)")
    print(f"{'phase (ends at)':18s} {'GPU ms':>8s} {'host ms':>8s} {'drained':>8s}")
    for n in ["forward", "backward", "prefetch", "optimizer", "end", "next-step start"]:
        if gpu[n]:
            g = sorted(gpu[n])[len(gpu[n]) // 2]
            h = sorted(host[n])[len(host[n]) // 2]
            print(f"{n:18s} {g:8.3f} {h:8.3f} {dr[n] / len(gpu[n]):8.2f}")


if __name__ == "__main__":
    main()
