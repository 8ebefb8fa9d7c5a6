"""Benchmark: adversarial-train frames/s of the SECOND KITTI step (BASELINE.json).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \\
        --master-port P bench.py --gpus N --steps K --warmup W

Workload = the metric's own config (BASELINE.json metric "SECOND KITTI-3class", configs[2]):
AdversarialVoxelNet (SECOND) KITTI 3-class (perturber hidden [64, 128, 64], 6 anchors per BEV
cell), batch 6 frames per GPU, perturber active (_epoch = 3), bf16 perf mode (fp32 voxelize /
perturber / sparse layer 0 / head losses; bf16 MFMA sparse layers 1-11 and SECOND/FPN), ClipAdamW
(clip 0.5 + AdamW), synthetic HDL-64E-like frames pre-staged in HBM. `--classes 1` is configs[1]
(Car-only). N > 1: frames sharded across ranks (weak scaling), DDP gradient all-reduce over RCCL.

`--gpus N` is honoured: under torch.distributed.run the world size must equal N (else exit 2);
a plain `python bench.py --gpus N` (N > 1) starts torch.distributed.run with N ranks as a child
process (before this process touches the GPU) and exits with its status. Rank 0 prints ONE JSON
line; `n_gpus` is the process-group world size.
"""
from __future__ import annotations

import argparse
import json
import os
import time

import numpy as np
import torch
import torch.distributed as dist


def _args():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=None, help="frames per GPU (6 KITTI, 4 nuScenes)")
    ap.add_argument("--classes", type=int, default=3, choices=[1, 3],
                    help="3 = KITTI 3-class (the metric's config, default); 1 = Car-only (BASELINE configs[1])")
    ap.add_argument("--model", default="voxelnet", choices=["voxelnet", "strong", "centerpoint"],
                    help="strong = StrongAdversarialVoxelNet, sensor_error_bound 0.4 (BASELINE config 5); "
                         "centerpoint = AdversarialCenterPoint nuScenes, batch 4 (BASELINE config 4)")
    ap.add_argument("--fp32", action="store_true", help="dense part in fp32 (parity mode)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-frames", type=int, default=2,
                    help="frames per CPU-baseline step (bounded sample: 3 warm-up + 5 timed steps)")
    ap.add_argument("--no-parity-mode", action="store_true",
                    help="skip the fp32 parity-mode timing that follows the headline (bf16) timing")
    ap.add_argument("--parity-steps", type=int, default=8)
    ap.add_argument("--roofline-kernel", default="dense",
                    help="'dense' (the dominant kernel: 3x3 stride-1 bf16 conv, rpc::dn::k_conv3x3<0>) or "
                         "op,ci,co of the sparse conv launches timed with HIP events")
    return ap.parse_args()


def _batches(n, B, rank, dev, classes):
    from robustpointclouds_amd.anchor_head import pack_gt
    from robustpointclouds_amd.synthetic import kitti_batch
    out = []
    for j in range(n):
        pts, boxes, labels = kitti_batch(B, seed0=(rank * n + j) * B, num_classes=classes)
        out.append(([torch.from_numpy(p).to(dev) for p in pts], _gt(boxes, labels, dev)))
    return out


def _nus_batches(n, B, rank, dev):
    """Synthetic 10-sweep nuScenes frames [N, 5] + 20-40 GT boxes [M, 9] per frame, padded on device."""
    from robustpointclouds_amd.center_head import pack_gt
    from robustpointclouds_amd.synthetic import nus_frame, nus_gt_boxes
    out = []
    for j in range(n):
        seeds = [(rank * n + j) * B + i for i in range(B)]
        pts = [torch.from_numpy(nus_frame(s)).to(dev) for s in seeds]
        gts = [nus_gt_boxes(s) for s in seeds]
        gb, gl = pack_gt([torch.from_numpy(b) for b, _ in gts], [torch.from_numpy(l) for _, l in gts], dev)
        out.append((pts, dict(gt_boxes=gb, gt_labels=gl)))
    return out


def _gt(boxes, labels, dev):
    from robustpointclouds_amd.anchor_head import pack_gt
    gb, gl = pack_gt(list(zip(boxes, labels)), dev)
    return dict(gt_boxes=gb, gt_labels=gl)


PEAK = {"fp32_mfma": 157.3, "bf16_mfma": 2500.0}   # TFLOP/s dense, MI355X_MICROARCH.md


def _traffic(kernel_tag, model="voxelnet"):
    """HBM bytes per launch of one kernel from the newest committed PMC summary of this model's step that has
    it (tools/pmc_traffic.py: FETCH_SIZE x 2 + WRITE_SIZE, KB -> bytes) and that summary's file name, else
    (None, None). `kernel_tag` is matched against the kernel's name without its argument list. Summaries are
    rNN_pmc_traffic_vMM.json (the SECOND steps: 3-class, Car, strong) or rNN_pmc_traffic_<model>_vMM.json
    (e.g. centerpoint): a kernel of the same name runs other shapes in another model's step."""
    import glob
    import re

    model = "centerpoint" if model == "centerpoint" else "voxelnet"

    def parse(f):   # newest round, then newest version (mtimes do not survive copies)
        m = re.search(r"r(\d+)_pmc_traffic_(?:([a-z]+)_)?v(\d+)", os.path.basename(f))
        return ((int(m.group(1)), int(m.group(3))), m.group(2) or "voxelnet") if m else ((-1, -1), "voxelnet")
    files = sorted((f for f in glob.glob(os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles",
                                                      "*pmc_traffic*.json")) if parse(f)[1] == model),
                   key=lambda f: parse(f)[0])
    # k_conv3x3y's data gradients with fused BatchNorm-backward sums are their own instantiation (<0, true>, r06):
    # "<0> +bnbwd" takes that one's traffic, the plain "<0>" the <0, false> one; other kernels' "+bnbwd" launches
    # share the plain kernel's name and have no traffic figure of their own
    bnb = kernel_tag.endswith(" +bnbwd")
    tag = kernel_tag[:-len(" +bnbwd")] if bnb else kernel_tag
    exact = [tag[:-1] + (", true>" if bnb else ", false>")] if tag.endswith(">") else []
    if not bnb:
        exact.append(tag)
    loose = tag[:-1] + "," if tag.endswith(">") and not bnb else None   # trailing template arguments omitted
    for f in reversed(files):
        d = json.load(open(f))
        ks = d.get("kernels", {})
        for name, v in ks.items():
            base = name.split("(")[0].strip()
            if base in exact or any(name.startswith(e + "(") for e in exact):
                return v.get("hbm_bytes_per_launch"), os.path.basename(f)
        for name, v in ks.items():
            base = name.split("(")[0].strip()
            if loose and base.startswith(loose):
                return v.get("hbm_bytes_per_launch"), os.path.basename(f)
    return None, None


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or "unknown"


def cpu_baseline(frames: int, classes: int, warmup: int = 3, steps: int = 5):
    """The oracle restatement of the whole step on the host cores (bounded sample; BASELINE.md §3:
    3 warm-up steps, >= 5 timed steps, CPU model and thread count reported)."""
    from oracle import anchor_head as oh
    from oracle import voxelize as ov
    from oracle.perturber import OraclePerturber, perturb_voxels
    from oracle.sparse_encoder import OracleSparseEncoder
    from robustpointclouds_amd.anchor_head import pack_gt
    from robustpointclouds_amd.plugin.models.adversarial.voxel_perturber import VoxelPerturber
    from robustpointclouds_amd.synthetic import KITTI_PC_RANGE, KITTI_VOXEL_SIZE, kitti_batch
    from robustpointclouds_amd.trainer import make_kitti_model
    cores = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    torch.set_num_threads(cores)
    model = make_kitti_model(num_classes=classes, device=None)  # CPU torch modules (dense part)
    adv = model.adversary
    lin = [m for m in adv.model if isinstance(m, torch.nn.Linear)]
    bns = [m for m in adv.model if isinstance(m, torch.nn.BatchNorm1d)]
    att = [m for m in adv.attention if isinstance(m, torch.nn.Linear)]
    w = {}
    for l, m in enumerate(lin):
        w[f"W{l}"], w[f"b{l}"] = m.weight.detach().numpy(), m.bias.detach().numpy()
    for l, m in enumerate(bns):
        w[f"g{l}"], w[f"be{l}"] = m.weight.detach().numpy(), m.bias.detach().numpy()
    for l, m in enumerate(att):
        w[f"Wa{l}"], w[f"ba{l}"] = m.weight.detach().numpy(), m.bias.detach().numpy()
    op = OraclePerturber(w, 4, adv.hidden_channels, dtype=torch.float32)
    enc = OracleSparseEncoder(model.middle_encoder, dtype=torch.float32)
    params = [t for t in op.p.values()] + [p for d in enc.params for p in (d["W"], d["g"], d["b"])] + \
        [p for n, p in model.named_parameters() if not n.startswith(("adversary", "middle_encoder"))]
    opt = torch.optim.AdamW(params, lr=1e-4, weight_decay=1e-3)
    pts, boxes, labels = kitti_batch(frames, seed0=1000, num_classes=classes)
    gt = pack_gt(list(zip(boxes, labels)), torch.device("cpu"))
    head = model.bbox_head
    hcfg = oh.cfg_of(head)
    gen = head.prior_generator
    anchors = oh.grid_anchors(200, 176, gen.ranges, gen.sizes, gen.rotations)

    def step():
        vox, coors, npts = ov.voxelize_frames(pts, KITTI_VOXEL_SIZE, KITTI_PC_RANGE, 5, 16000)
        vfe, _, ld = perturb_voxels(op, vox, npts)
        x = enc.forward(vfe.float(), coors, frames)
        x = model.neck(model.backbone(x))
        w, b = head._stacked()
        ref = oh.head_losses_from_z(hcfg, torch.nn.functional.conv2d(x[0], w), b, anchors, gt[0], gt[1])
        losses = {k: [ref[k]] for k in ("loss_cls", "loss_bbox", "loss_dir")}
        total = sum(v[0] for v in losses.values()) + 0.01 * (3 * ld["intensity_loss"] + 10 * ld["bias_loss"] +
                                                             10 * ld["imbalance_loss"]) + 0.02 * ld["l2_norm"]
        total.backward()
        torch.nn.utils.clip_grad_norm_(params, 0.5)
        opt.step()
        opt.zero_grad()

    for _ in range(warmup):
        step()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    dt = time.perf_counter() - t0
    return dict(value=round(frames * steps / dt, 4), unit="frames/s", cores=cores, kind="port",
                cpu_model=_cpu_model(), warmup=warmup, steps=steps,
                sample=f"{steps} timed steps (after {warmup} warm-up) of the oracle restatement (C voxelize, "
                       f"torch-CPU fp32 perturber + sparse encoder, torch-CPU SECOND/FPN/Anchor3DHead fwd+bwd, "
                       f"AdamW), {frames} synthetic KITTI frames per step, {classes}-class, {dt:.1f} s timed")


def _dense_flops_per_frame(model, H, W):
    """Algorithmic FLOPs of one frame through SECOND + SECONDFPN + the head's 1x1 convs: forward, data
    gradient and weight gradient of every conv (3 x 2·MACs; the first conv's data gradient is the BEV
    gradient the sparse encoder needs), from the modules' own shapes."""
    from torch import nn
    total = 0.0
    h, w = H, W
    dims = []
    for blk in model.backbone.blocks:
        for m in blk:
            if isinstance(m, nn.Conv2d):
                s = m.stride[0]
                h, w = (h + s - 1) // s, (w + s - 1) // s
                total += 3 * 2.0 * h * w * m.in_channels * m.out_channels * m.kernel_size[0] * m.kernel_size[1]
        dims.append((h, w))
    for (hi, wi), d in zip(dims, model.neck.deblocks):
        m = d[0]
        total += 3 * 2.0 * hi * wi * m.in_channels * m.out_channels * m.kernel_size[0] * m.kernel_size[1]
    head = model.bbox_head
    for c in head._convs():
        total += 3 * 2.0 * H * W * c.in_channels * c.out_channels
    return total


def _perf_kernel_dtype():
    """The perf mode's operand formats, read from the modules that choose them."""
    from robustpointclouds_amd import sparse_encoder as se
    fwd = "fp16" if se.FWD_FMT == 1 else "bf16"
    return (f"fp32 voxelize / sparse layer 0 / head losses; perturber hidden layers fp32 MFMA (weight gradient "
            f"split-bf16); sparse layers 1-11 on MFMA with {fwd} forward operands and bf16 backward (dz) operands "
            f"(fp32 accumulate, fp32 BN statistics); SECOND/FPN/head convs bf16 MFMA (fp32 accumulate)")


def _perturber_flops_per_point(adv):
    from torch import nn
    lin = [m for m in list(adv.model) + list(adv.attention or []) if isinstance(m, nn.Linear)]
    return 3 * 2.0 * sum(m.in_features * m.out_features for m in lin)


def _perturber_stages(stages, n_valid, adv, peak):
    """The perturber stages against the fp32 MFMA roof: its hidden layers are fp32 MFMA GEMMs over the
    valid points (2·C_in·C_out FLOP per point per Linear forward, twice that backward: data + weight
    gradient), so FLOP/s over the stage's HIP-event time is the figure that characterises it (its
    compulsory HBM bytes — voxels in, perturbed voxels out — ignore the activation traffic that bounds it)."""
    out = {}
    fwd_pp = _perturber_flops_per_point(adv) / 3.0
    for name, mult in (("perturber_fwd", 1.0), ("perturber_bwd", 2.0)):
        st = (stages or {}).get(name)
        if not st or n_valid <= 0:
            continue
        fl = mult * fwd_pp * n_valid
        tf = fl / (st["avg_ms"] * 1e-3) / 1e12
        out[name] = dict(bound="mfma", flops_per_launch=round(fl), avg_ms=st["avg_ms"], achieved=round(tf, 2),
                         peak=peak, unit="TFLOP/s", frac=round(tf / peak, 4), valid_points=int(n_valid),
                         work="2*C_in*C_out FLOP per valid point per Linear layer (x1 forward, x2 backward)")
    return out


def _parity_mode(a, data, ready, dev, nus, fpf):
    """The reference's own precision on the same frames: the metric's config trains fp32
    (configs/adversarial/adversarial-second_hv_secfpn_8xb6-80e_kitti-3d-3class.py:130-131, type
    'OptimWrapper'). A fresh model (same seed) in the fp32 parity mode — fp32 perturber, fp32 sparse
    encoder, SECOND / FPN / head on the fp32-MFMA engine — the mode the 1e-4 parity tests cover, timed
    like the headline: warm-up, then K steps between barrier + synchronize, max over ranks."""
    from robustpointclouds_amd import stage_timer
    from robustpointclouds_amd.trainer import Trainer, make_kitti_model, make_nus_model
    torch.manual_seed(0)
    model = (make_nus_model(device=dev, epoch=3) if nus else
             make_kitti_model(num_classes=a.classes, device=dev, epoch=3, variant=a.model))
    tr = Trainer(model, ddp=dist.is_initialized(), bf16=False, device=dev)
    NB, W, K = len(data), 3, a.parity_steps
    for i in range(W):
        tr.train_step(*data[i % NB], next_points=data[(i + 1) % NB][0], next_ready=ready)
    torch.cuda.synchronize()
    if dist.is_initialized():
        dist.barrier()
    t0 = time.perf_counter()
    for i in range(K):
        tr.train_step(*data[i % NB], next_points=data[(i + 1) % NB][0], next_ready=ready)
    torch.cuda.synchronize()
    if dist.is_initialized():
        dist.barrier()
    dt = time.perf_counter() - t0
    # one more (eager) step with the stage timers on, for the perturber's fp32-MFMA figure
    stage_timer.TIMER.reset()
    stage_timer.TIMER.enabled = True
    tr.train_step(*data[K % NB], next_points=data[(K + 1) % NB][0], next_ready=ready)
    torch.cuda.synchronize()
    stage_timer.TIMER.enabled = False
    stages = stage_timer.TIMER.summary()
    stage_timer.TIMER.reset()
    flags = getattr(model, "_last_flags", None)
    n_valid = float(flags[4].item()) if flags is not None else 0.0
    if dist.is_initialized():
        t = torch.tensor([dt], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    world = dist.get_world_size() if dist.is_initialized() else 1
    fps = world * a.batch * K / dt
    res = dict(dtype="fp32", frames_per_s=round(fps, 3), ms_per_step=round(1000 * dt / K, 3), steps=K, warmup=W,
               kernel_dtype="fp32 end to end: voxelize, perturber (fp32 MFMA), sparse encoder, SECOND/FPN and "
                            "head GEMMs on v_mfma_f32_16x16x4_f32, fp32 losses")
    if fpf:
        ach = fps / world * fpf / 1e12
        res["step_roofline"] = dict(bound="mfma", flop_per_frame=round(fpf), achieved=round(ach, 2),
                                    peak=PEAK["fp32_mfma"], unit="TFLOP/s", frac=round(ach / PEAK["fp32_mfma"], 4),
                                    work="the headline's algorithmic FLOPs per frame (dense + sparse + perturber, "
                                         "forward + data gradient + weight gradient) per GPU")
    if stages:
        res["stage_roofline"] = dict(bound="hbm", unit="GB/s",
                                     stages={k: v for k, v in stages.items() if not k.startswith("perturber")})
    if model.__dict__.get("adversary") is not None or getattr(model, "adversary", None) is not None:
        res["perturber_roofline"] = _perturber_stages(stages, n_valid, model.adversary, PEAK["fp32_mfma"])
    del tr, model
    torch.cuda.empty_cache()
    return res


def _launch_ranks(n: int) -> int:
    """Re-run this script under torch.distributed.run with n ranks (child process; no GPU touched
    here) and return its exit status."""
    import socket
    import subprocess
    import sys
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__), *sys.argv[1:]]
    return subprocess.run(cmd, env=env).returncode


def main():
    a = _args()
    import sys
    if "RANK" not in os.environ and a.gpus > 1:
        sys.exit(_launch_ranks(a.gpus))
    from robustpointclouds_amd.trainer import Trainer, init_distributed, make_kitti_model, make_nus_model
    rank, world, local = init_distributed()
    if world != a.gpus:
        print(json.dumps(dict(error=f"--gpus {a.gpus} but the process group has {world} ranks")), flush=True)
        sys.exit(2)
    # init_distributed picked the device (local rank modulo the visible GPUs)
    dev = torch.device("cuda", torch.cuda.current_device())
    torch.cuda.set_device(dev)
    torch.manual_seed(0)
    nus = a.model == "centerpoint"
    if a.batch is None:
        a.batch = 4 if nus else 6
    if nus:
        model = make_nus_model(device=dev, epoch=3)
    else:
        model = make_kitti_model(num_classes=a.classes, device=dev, epoch=3, variant=a.model)
    tr = Trainer(model, ddp=dist.is_initialized(), bf16=not a.fp32, device=dev)
    from robustpointclouds_amd import dense_bev
    from robustpointclouds_amd.sparse_encoder import KernelTimer
    sparse_timer = None
    if a.roofline_kernel == "dense":
        timer = dense_bev.ConvTimer()
        dense_bev.TIMER = timer
        op = ci = co = None
        # every sparse conv launch too (forward, data and weight gradients): the roofline entry is the MFMA
        # kernel with the most time per step across dense and sparse (config 4's is sparse)
        if getattr(model, "middle_encoder", None) is not None:
            sparse_timer = KernelTimer()
            model.middle_encoder.timer = sparse_timer
    else:
        op, ci, co = a.roofline_kernel.split(",")
        timer = KernelTimer(op, int(ci), int(co))
        model.middle_encoder.timer = timer
    NB = 4
    data = _nus_batches(NB, a.batch, rank, dev) if nus else _batches(NB, a.batch, rank, dev, a.classes)
    # the synthetic frames are staged in HBM once: the batch prefetch need not wait for anything to read them
    ready = torch.cuda.Event()
    ready.record(torch.cuda.current_stream(dev))
    # each step queues the next step's hard voxelisation on a side stream (Trainer.train_step
    # next_points): the timed region still voxelises K batches, one per step. The dense part replays
    # HIP graphs from the second step on (dense_bev.GRAPHS).
    for i in range(a.warmup):
        tr.train_step(*data[i % NB], next_points=data[(i + 1) % NB][0], next_ready=ready)
    torch.cuda.synchronize()
    if dist.is_initialized():
        dist.barrier()
    t0 = time.perf_counter()
    for i in range(a.steps):
        tr.train_step(*data[i % NB], next_points=data[(i + 1) % NB][0], next_ready=ready)
    torch.cuda.synchronize()
    if dist.is_initialized():
        dist.barrier()
    dt = time.perf_counter() - t0
    # per-launch HIP-event timing of the roofline kernels: ROCm cannot record timing events inside a captured
    # graph, so 2 more steps of the same workload run with the dense graphs off and the kernel timers on (same
    # kernels, shapes and inputs as the timed steps; rocprof summaries under profiles/ agree); the second of
    # them also counts the step's algorithmic FLOPs. The HBM-bound stages are timed in 2 further steps of their
    # own (dense graphs on, as in the timed loop), so no per-launch event pair of the kernel timers falls inside
    # a stage's event pair (the per-sparse-launch events had inflated sparse_fwd / sparse_bwd)
    from robustpointclouds_amd import stage_timer
    graphs = dense_bev.GRAPHS
    dense_bev.GRAPHS = False
    timer.enabled = True
    if sparse_timer is not None:
        sparse_timer.enabled = True
    me = getattr(model, "middle_encoder", None)
    for i in range(a.steps, a.steps + 2):
        if i == a.steps + 1 and me is not None:
            me.flop_probe = []
        tr.train_step(*data[i % NB], next_points=data[(i + 1) % NB][0], next_ready=ready)
    torch.cuda.synchronize()
    timer.enabled = False
    if sparse_timer is not None:
        sparse_timer.enabled = False
    dense_bev.GRAPHS = graphs
    stage_timer.TIMER.enabled = True
    for i in range(a.steps + 2, a.steps + 4):
        tr.train_step(*data[i % NB], next_points=data[(i + 1) % NB][0], next_ready=ready)
    torch.cuda.synchronize()
    stage_timer.TIMER.enabled = False
    ks = timer.summary()
    sks = sparse_timer.per_kernel() if sparse_timer is not None else {}
    stages = stage_timer.TIMER.summary()
    step_flops = None
    if me is not None and me.flop_probe and not nus:
        sparse = sum(3 * 2.0 * float((nbr >= 0).sum().item()) * ci * co for nbr, ci, co in me.flop_probe[-1])
        me.flop_probe = None
        flags = getattr(model, "_last_flags", None)
        n_valid = float(flags[4].item()) if flags is not None else 0.0
        pert = n_valid * _perturber_flops_per_point(model.adversary) if model.adversary is not None else 0.0
        dense = _dense_flops_per_frame(model, 200, 176) * a.batch
        step_flops = dict(dense=dense, sparse=sparse, perturber=pert, total=dense + sparse + pert)
    if dist.is_initialized():
        t = torch.tensor([dt], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    n_valid = 0.0
    if step_flops is not None:
        n_valid = step_flops["perturber"] / _perturber_flops_per_point(model.adversary) if model.adversary is not None \
            else 0.0
    # the reference's precision (fp32) on the same frames, after the headline timing (all ranks take part)
    parity = None
    if not a.fp32 and not a.no_parity_mode and a.roofline_kernel == "dense":
        fpf = step_flops["total"] / a.batch if step_flops is not None else None
        parity = _parity_mode(a, data, ready, dev, nus, fpf)
    frames = world * a.batch * a.steps
    if rank == 0:
        metric = ("adversarial-train frames/sec/GPU, CenterPoint nuScenes 10-class (BASELINE config 4)" if nus else
                  "adversarial-train frames/sec/GPU, StrongAdversarialVoxelNet KITTI (BASELINE config 5, not the "
                  "metric)" if a.model != "voxelnet" else
                  "adversarial-train frames/sec/GPU, SECOND KITTI-3class, at 1/2/4/8 MI355X" if a.classes == 3 else
                  "adversarial-train frames/sec/GPU, SECOND KITTI Car-only (BASELINE configs[1], not the metric)")
        workload = ("AdversarialCenterPoint nuScenes 10-class (voxel 0.1 m, 10-sweep HDL-32E-like frames, "
                    "basicblock SparseEncoder, SECOND/FPN, DCN CenterHead)" if nus else
                    ("AdversarialVoxelNet" if a.model == "voxelnet" else
                     "StrongAdversarialVoxelNet (sensor_error_bound 0.4, config 5)") +
                    " (SECOND) KITTI " + ("Car-only" if a.classes == 1 else "3-class"))
        res = dict(metric=metric,
                   value=round(frames / dt, 3), unit="frames/s", n_gpus=world, steps=a.steps, warmup=a.warmup,
                   ms_per_step=round(1000 * dt / a.steps, 3), higher_is_better=True, scaling="weak",
                   vs_baseline=None, dtype="fp32" if a.fp32 else "bf16", data="synthetic",
                   config=dict(workload=workload + f", batch {a.batch}/GPU, perturber active (_epoch=3)",
                               global_batch=world * a.batch, frames_per_gpu=a.batch,
                               dense_dtype="fp32" if a.fp32 else "bf16",
                               kernel_dtype=("fp32 (voxelize, perturber, sparse encoder)" if a.fp32 else
                                             _perf_kernel_dtype()),
                               parallelism=f"dp{world}",
                               dist_backend=dist.get_backend() if dist.is_initialized() else None))
        if ks and op is None:
            # one entry per kernel, each over its own launches with its own FLOPs / bytes / PMC traffic;
            # `roofline` is the one with the most time per step
            peak = PEAK["fp32_mfma"] if a.fp32 else PEAK["bf16_mfma"]
            ents = []
            for name, k in ks.items():
                tr_bytes, tr_src = _traffic(name, a.model)
                ents.append(dict(bound="mfma", kernel=name, achieved=round(k["tflops"], 3), peak=peak, unit="TFLOP/s",
                                 frac=round(k["tflops"] / peak, 4), traffic=tr_bytes, traffic_source=tr_src,
                                 avg_launch_ms=round(k["avg_ms"], 4), launches=k["launches"],
                                 flops_per_launch=k["flops_per_launch"],
                                 algorithmic_bytes_per_launch=k["bytes_per_launch"],
                                 achieved_gbps=round(k["gbps"], 1), ms_per_step=round(k["total_ms"] / 2, 4),
                                 work="2*B*H*W*C_in*C_out*9 FLOP per launch (SECOND 3x3 stride-1 conv, "
                                      "forward + flipped-tap data gradient)"))
            ents.sort(key=lambda e: -e["ms_per_step"])
            for e in ents:
                if e["kernel"].endswith("+bnbwd"):
                    e["work"] += "; data gradient through rpc_dense_conv_bnbwd: the epilogue also reads the " \
                                 "next layer's pre-activation image (in the bytes) for its BatchNorm-backward sums"
            # headline: each S1 kernel over ALL its launches — plain forward / data gradient and
            # the fused-epilogue data gradients (rpc_dense_conv_bnbwd) together: total FLOPs / total HIP-event
            # time; the per-variant entries stay in roofline_kernels
            comb = {}
            for e in ents:
                base = e["kernel"].replace(" +bnbwd", "")
                c = comb.setdefault(base, dict(flops=0.0, ms=0.0, launches=0, bytes=0.0, tr=0.0, tr_n=0, srcs=set()))
                c["flops"] += e["flops_per_launch"] * e["launches"]
                c["ms"] += e["avg_launch_ms"] * e["launches"]
                c["launches"] += e["launches"]
                c["bytes"] += e["algorithmic_bytes_per_launch"] * e["launches"]
                if e["traffic"] is not None:
                    c["tr"] += e["traffic"] * e["launches"]
                    c["tr_n"] += e["launches"]
                    c["srcs"].add(e["traffic_source"])
            alls = []
            for base, c in comb.items():
                tf = c["flops"] / (c["ms"] * 1e-3) / 1e12
                alls.append(dict(bound="mfma", kernel=base + " (all launches)", achieved=round(tf, 3), peak=peak,
                                 unit="TFLOP/s", frac=round(tf / peak, 4),
                                 traffic=(c["tr"] / c["tr_n"]) if c["tr_n"] else None,
                                 traffic_source=(", ".join(sorted(c["srcs"])) +
                                                 (f" (PMC for {c['tr_n']} of {c['launches']} launches)"
                                                  if c["tr_n"] < c["launches"] else "")) if c["tr_n"] else None,
                                 avg_launch_ms=round(c["ms"] / c["launches"], 4), launches=c["launches"],
                                 flops_per_launch=c["flops"] / c["launches"],
                                 algorithmic_bytes_per_launch=c["bytes"] / c["launches"],
                                 ms_per_step=round(c["ms"] / 2, 4),
                                 work="2*B*H*W*C_in*C_out*9 FLOP per launch over every launch of the kernel "
                                      "(forward, data gradient, fused-epilogue data gradient)"))
            # the sparse conv kernels (HIP events per launch; FLOPs from the valid rulebook pairs)
            for name, k in sks.items():
                pk = PEAK["bf16_mfma"] if k["dtype"] == "bf16" else PEAK["fp32_mfma"]
                tr_bytes, tr_src = _traffic(name, a.model)
                alls.append(dict(bound="mfma", kernel=name, achieved=round(k["tflops"], 3), peak=pk, unit="TFLOP/s",
                                 frac=round(k["tflops"] / pk, 4), traffic=tr_bytes, traffic_source=tr_src,
                                 avg_launch_ms=round(k["avg_ms"], 4), launches=k["launches"],
                                 flops_per_launch=k["flops_per_launch"], ms_per_step=round(k["total_ms"] / 2, 4),
                                 work="2*C_in*C_out FLOP per valid rulebook pair (sparse conv, " + k["dtype"] +
                                      " MFMA; timed in the per-layer backward loop" +
                                      ("; a weight gradient's time includes its fixed-order slab reduce, launched by "
                                       "the same C-ABI call" if "wgrad" in name else "") + ")"))
            alls.sort(key=lambda e: -e["ms_per_step"])
            res["roofline"] = dict(alls[0])
            res["roofline_kernels"] = alls + ents
        elif ks:
            peak = PEAK["bf16_mfma" if ks["dtype"] == "bf16" else "fp32_mfma"]
            tag = ks["kernel"]
            res["roofline"] = dict(bound="mfma", achieved=round(ks["tflops"], 3), peak=peak,
                                   unit="TFLOP/s", frac=round(ks["tflops"] / peak, 4),
                                   traffic=_traffic(tag, a.model)[0],
                                   kernel=f"{tag} (sparse conv {op} {ci}->{co}, {ks['dtype']} MFMA)",
                                   avg_launch_ms=round(ks["avg_ms"], 4),
                                   flops_per_launch=ks["flops_per_launch"], launches=ks["launches"],
                                   work="2*C_in*C_out FLOP per valid rulebook pair")
        if stages:
            # HBM-bound stages: compulsory bytes (stage_timer.py) / HIP-event time / 8 TB/s. The perturber is not
            # one (its fp32 activations, not its voxels, are its traffic): its stages are in perturber_roofline
            res["stage_roofline"] = dict(bound="hbm", unit="GB/s", timed_apart_from_kernel_timers=True,
                                         stages={k: v for k, v in stages.items() if not k.startswith("perturber")})
        if step_flops is not None:
            # whole-step algorithmic FLOP rate, the per-frame constant counted on this run's
            # synthetic frames: dense convs from the module shapes, sparse convs from the valid rulebook pairs,
            # perturber from the valid points (each x3: forward, data gradient, weight gradient)
            fpf = step_flops["total"] / a.batch
            res["step_roofline"] = dict(flop_per_frame=round(fpf), flop_per_frame_split={
                k: round(v / a.batch) for k, v in step_flops.items() if k != "total"},
                achieved=round(frames / dt * fpf / 1e12, 1), peak=PEAK["fp32_mfma" if a.fp32 else "bf16_mfma"], unit="TFLOP/s",
                frac=round(frames / dt * fpf / 1e12 / PEAK["fp32_mfma" if a.fp32 else "bf16_mfma"], 4))
        if stages and step_flops is not None and model.adversary is not None:
            res["perturber_roofline"] = _perturber_stages(stages, n_valid, model.adversary, PEAK["fp32_mfma"])
        if parity is not None:
            res["parity_mode"] = parity
        if not a.no_cpu_baseline and a.model == "voxelnet":
            res["cpu_baseline"] = cpu_baseline(a.cpu_frames, a.classes)
        print(json.dumps(res), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
