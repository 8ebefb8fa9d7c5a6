"""Multi-process check of the data-parallel step on the GPU (run under torch.distributed.run).

    RPC_DIST_BACKEND=gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \\
        --master-addr 127.0.0.1 --master-port 29611 tools/ddp_check.py

    python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
        --master-addr 127.0.0.1 --master-port 29611 tools/ddp_check.py     # nccl = RCCL, one rank

Each rank trains the real KITTI 3-class model (the metric's config; RPC_DDP_CLASSES=1 for Car)
in bf16 perf mode (HIP kernels, ClipAdamW) on its own frames. First one DDP forward / backward: the
gradients DDP leaves in .grad must equal, on rank 0, the average of the per-rank gradients of a
single-process reference model (same initial weights) run on each rank's frames in turn (relative
L2 <= 1e-6 per parameter: only the averaging arithmetic differs). Then 3 training steps under DDP;
afterwards every parameter must be bit-identical across ranks (the gradient all-reduce and the
optimizer see the same averaged gradients) and the losses finite. With gloo several ranks may share one GPU (the
1-GPU test box); without RPC_DIST_BACKEND the backend is nccl (RCCL), one rank per GPU."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch
import torch.distributed as dist


def _frames(rank, step, classes, dev):
    from robustpointclouds_amd.anchor_head import pack_gt
    from robustpointclouds_amd.synthetic import kitti_batch
    pts, boxes, labels = kitti_batch(2, seed0=100 * rank + 10 * step, num_classes=classes)
    gb, gl = pack_gt(list(zip(boxes, labels)), dev)
    return [torch.from_numpy(p).to(dev) for p in pts], dict(gt_boxes=gb, gt_labels=gl)


def _grads_of(module, loss_fn):
    from robustpointclouds_amd.adversarial_loss import parse_losses
    with torch.autocast("cuda", dtype=torch.bfloat16):
        losses = loss_fn()
    parse_losses(losses)[0].backward()
    g = [None if p.grad is None else p.grad.detach().clone() for p in module.parameters()]
    for p in module.parameters():
        p.grad = None
    return g


def _averaged_gradient_check(tr, model, rank, world, dev, classes):
    """One DDP forward / backward vs the average of single-process per-rank gradients (rank 0)."""
    from robustpointclouds_amd.trainer import make_kitti_model
    pts, gt = _frames(rank, 0, classes, dev)

    def ddp_loss():
        batch = model.data_preprocessor(dict(inputs=dict(points=pts)), training=True)["inputs"]
        return tr.model(batch, gt, mode="loss")
    model.train()
    g_ddp = _grads_of(model, ddp_loss)
    ok, worst = True, 0.0
    if rank == 0:
        torch.manual_seed(0)
        ref = make_kitti_model(num_classes=classes, device=dev, epoch=3)
        ref.load_state_dict(model.state_dict())
        from robustpointclouds_amd.trainer import Trainer
        Trainer._select_engines(ref, True)
        ref.train()
        acc = None
        for r in range(world):
            p_r, gt_r = _frames(r, 0, classes, dev)

            def ref_loss():
                batch = ref.data_preprocessor(dict(inputs=dict(points=p_r)), training=True)["inputs"]
                return ref.loss(batch, gt_r)
            g = _grads_of(ref, ref_loss)
            acc = g if acc is None else [a if b is None else (b if a is None else a + b) for a, b in zip(acc, g)]
        for a, b in zip(g_ddp, acc):
            if a is None or b is None:
                ok = ok and (a is None) == (b is None)
                continue
            b = b / world
            rel = float((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30))
            worst = max(worst, rel)
        ok = ok and worst <= 1e-6
    flag = torch.tensor([1 if ok else 0], device=dev)
    dist.broadcast(flag, 0)
    return bool(flag.item()), worst


def main():
    from robustpointclouds_amd.anchor_head import pack_gt
    from robustpointclouds_amd.synthetic import kitti_batch
    from robustpointclouds_amd.trainer import Trainer, init_distributed, make_kitti_model
    rank, world, local = init_distributed()
    dev = torch.device("cuda", torch.cuda.current_device())
    torch.manual_seed(0)
    classes = int(os.environ.get("RPC_DDP_CLASSES", "3"))
    model = make_kitti_model(num_classes=classes, device=dev, epoch=3)
    tr = Trainer(model, ddp=True, bf16=True, device=dev)
    assert isinstance(tr.model, torch.nn.parallel.DistributedDataParallel)
    losses = []
    batches = []
    for step in range(3):
        pts, boxes, labels = kitti_batch(2, seed0=100 * rank + 10 * step, num_classes=classes)
        gb, gl = pack_gt(list(zip(boxes, labels)), dev)
        batches.append(([torch.from_numpy(p).to(dev) for p in pts], dict(gt_boxes=gb, gt_labels=gl)))
    avg_ok, worst = _averaged_gradient_check(tr, model, rank, world, dev, classes)
    for step in range(3):
        # as bench.py: the next batch is voxelised on a side stream during this step (Trainer prefetch)
        nxt = batches[step + 1][0] if step + 1 < len(batches) else None
        lg = tr.train_step(*batches[step], next_points=nxt)
        losses.append(float(sum(v for k, v in lg.items() if "loss" in k)))
    torch.cuda.synchronize()
    flat = torch.cat([p.detach().double().flatten() for p in model.parameters()])
    sums = torch.stack([flat.sum(), flat.abs().sum(), (flat * torch.arange(flat.numel(), device=dev,
                                                                             dtype=torch.float64)).sum()])
    allsums = [torch.zeros_like(sums) for _ in range(world)]
    dist.all_gather(allsums, sums)
    same = all(torch.equal(allsums[0], a) for a in allsums)
    # the collective itself: all_reduce(SUM) of rank+1 over the group's backend
    probe = torch.full((1 << 20,), float(rank + 1), device=dev)
    dist.all_reduce(probe)
    coll_ok = bool((probe == world * (world + 1) / 2).all())
    same = same and coll_ok
    ok = same and avg_ok and all(torch.isfinite(torch.tensor(l)) for l in losses)
    if rank == 0:
        print(json.dumps(dict(ddp="ok" if ok else "MISMATCH", world=world, backend=dist.get_backend(),
                              classes=classes, losses=losses, params_identical=same, all_reduce_ok=coll_ok,
                              averaged_grads_ok=avg_ok, averaged_grads_worst_rel=worst)),
              flush=True)
    dist.barrier()
    dist.destroy_process_group()
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
