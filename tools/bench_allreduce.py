#!/usr/bin/env python
"""RCCL all-reduce sweep for choosing the gradient bucket cap, wire dtype and RCCL channel/algorithm settings on
an MI355X node (7 point-to-point xGMI links per GPU, a ring drives one of them per channel).

    python tools/bench_allreduce.py --gpus 8                  # all configs, one torchrun per RCCL env setting
    python tools/bench_allreduce.py --gpus 8 --channels 4,8,16,32 --algos Ring,Tree

For every RCCL setting (NCCL_MIN_NCHANNELS / NCCL_MAX_NCHANNELS, NCCL_ALGO — read by RCCL at communicator
creation, hence one launch per setting) rank 0 prints JSON lines:
  * "size": one all-reduce of S MB (f32 and bf16): time, algorithm bandwidth, bus bandwidth 2(N-1)/N * S / t;
  * "buckets": the ResNet-50 gradient arena (25.56 M f32) cut at a bucket cap and issued back to back as async
    all-reduces, the way GradientBucketer issues them during backward: total time for the whole arena.
"""
import argparse
import itertools
import json
import os
import socket
import subprocess
import sys
import time

RESNET50_PARAMS = 25_557_032


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def worker(args):
    import torch
    import torch.distributed as dist
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    local = int(os.environ.get("LOCAL_RANK", rank))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist.init_process_group("nccl", device_id=dev)
    tag = {"channels": os.environ.get("NCCL_MAX_NCHANNELS", "default"), "algo": os.environ.get("NCCL_ALGO", "default"),
           "n_gpus": world}

    def timed(fn, iters):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(iters):
            fn()
        torch.cuda.synchronize()
        t = torch.tensor([(time.perf_counter() - t0) / iters], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    for mb in [float(x) for x in args.sizes.split(",")]:
        for dt in (torch.float32, torch.bfloat16):
            n = int(mb * (1 << 20)) // (4 if dt == torch.float32 else 2)
            x = torch.ones(n, dtype=dt, device=dev)
            t = timed(lambda: dist.all_reduce(x), args.iters)
            nbytes = x.numel() * x.element_size()
            if rank == 0:
                print(json.dumps(dict(tag, kind="size", mb=mb, dtype=str(dt).split(".")[-1], ms=round(t * 1e3, 4),
                                      algbw_gbs=round(nbytes / t / 1e9, 2),
                                      busbw_gbs=round(2 * (world - 1) / world * nbytes / t / 1e9, 2))), flush=True)
    for dt in (torch.float32, torch.bfloat16):
        arena = torch.ones(RESNET50_PARAMS, dtype=dt, device=dev)
        for cap in [float(x) for x in args.caps.split(",")]:
            step = max(1, int(cap * (1 << 20)) // arena.element_size())
            views = [arena[i:i + step] for i in range(0, arena.numel(), step)]

            def bucketed():
                works = [dist.all_reduce(v, async_op=True) for v in views]
                for w in works:
                    w.wait()
            t = timed(bucketed, max(5, args.iters // 2))
            if rank == 0:
                print(json.dumps(dict(tag, kind="buckets", cap_mb=cap, buckets=len(views), dtype=str(dt).split(".")[-1],
                                      ms=round(t * 1e3, 4),
                                      busbw_gbs=round(2 * (world - 1) / world * arena.numel() * arena.element_size()
                                                      / t / 1e9, 2))), flush=True)
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=8)
    ap.add_argument("--channels", default="default,8,16,32")
    ap.add_argument("--algos", default="default,Ring,Tree")
    ap.add_argument("--sizes", default="1,4,16,32,64,128,256")
    ap.add_argument("--caps", default="4,8,16,32,64,128")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--worker", action="store_true")
    args = ap.parse_args()
    if args.worker:
        return worker(args)
    rc = 0
    for ch, algo in itertools.product(args.channels.split(","), args.algos.split(",")):
        env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
        for k in ("NCCL_MIN_NCHANNELS", "NCCL_MAX_NCHANNELS", "NCCL_ALGO"):
            env.pop(k, None)
        if ch != "default":
            env["NCCL_MIN_NCHANNELS"] = env["NCCL_MAX_NCHANNELS"] = ch
        if algo != "default":
            env["NCCL_ALGO"] = algo
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
               "--master-addr", "127.0.0.1", "--master-port", str(_port()), os.path.abspath(__file__), "--worker",
               "--sizes", args.sizes, "--caps", args.caps, "--iters", str(args.iters)]
        r = subprocess.run(cmd, env=env, timeout=600)
        rc = rc or r.returncode
    return rc


if __name__ == "__main__":
    sys.exit(main())
