#!/usr/bin/env python
"""Headline benchmark: ResNet-50 v1.5 bf16 training throughput (images/sec, whole job).

Contract (driver): ``python bench.py --gpus N --steps K --warmup W``; for N>1 it is
launched under ``torch.distributed.run`` with one rank per GPU (RCCL over xGMI).
Per-GPU batch is fixed (weak scaling); the timed region holds exactly K full
training steps — device-side input conversion, forward, loss, backward with the
bucketed all-reduce, and the fused SGD-momentum update — bracketed by a barrier
and ``torch.cuda.synchronize()``; the max over ranks is reported by rank 0 as
one JSON line. Data: one synthetic ImageNet batch (random 224x224x3 f32 images,
random labels) resident on each GPU; weights random-init.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=256, help="per-GPU batch")
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--lr", type=float, default=0.1)
    ap.add_argument("--bucket-mb", type=float, default=None)
    ap.add_argument("--profile-steps", type=int, default=0)
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    import distributed_tensorflow_amd as dtf
    from distributed_tensorflow_amd import parallel
    from distributed_tensorflow_amd.data import synthetic_imagenet
    from distributed_tensorflow_amd.keras import losses, optimizers
    from distributed_tensorflow_amd.models import ResNet

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        if args.gpus > 1 and world == 1:
            print(f"bench.py: --gpus {args.gpus} needs a torch.distributed.run launch with {args.gpus} ranks",
                  file=sys.stderr)
            return 2
    strategy = parallel.MirroredStrategy(bucket_mb=args.bucket_mb)
    rank = strategy.worker_index
    dev = strategy.device
    depth = {"resnet50": 50, "resnet101": 101, "resnet152": 152}[args.model]

    with strategy.scope():
        model = ResNet(depth, num_classes=1000)
        model.compile(optimizer=optimizers.SGD(args.lr, momentum=0.9),
                      loss=losses.SparseCategoricalCrossentropy(from_logits=True))
    data = iter(synthetic_imagenet(args.batch, dev, seed=1234 + rank))

    def step():
        x, y = next(data)
        return model.train_step((x, y))

    for _ in range(args.warmup):
        logs = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        logs = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    loss = float(logs["loss"])
    t = torch.tensor([dt], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt = float(t.item())
    ms = dt / args.steps * 1e3
    global_batch = args.batch * world
    ips = global_batch * args.steps / dt
    if rank == 0:
        with open(os.path.join(ROOT, "BASELINE.json")) as f:
            base = json.load(f)
        pub = base.get("published") or {}
        ref = pub.get("resnet50_images_per_sec") if isinstance(pub, dict) else None
        out = {
            "metric": base["metric"],
            "value": round(ips, 2),
            "unit": "images/sec",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": (ips / ref) if ref else None,
            "dtype": "bf16",
            "data": "synthetic (random 224x224x3 images + labels resident on GPU; random-init weights)",
            "config": {"model": f"ResNet-{depth} v1.5", "global_batch": global_batch, "per_gpu_batch": args.batch,
                       "image_size": 224, "seq_len": None, "parallelism": f"dp{world}",
                       "strategy": "MirroredStrategy (1 process/GPU, RCCL)", "optimizer": "SGD momentum 0.9",
                       "final_loss": round(loss, 4)},
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
