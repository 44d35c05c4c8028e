#!/usr/bin/env python
"""Headline benchmark: ResNet-50 v1.5 bf16 training throughput (images/sec, whole job).

Contract (driver): ``python bench.py --gpus N --steps K --warmup W``; for N>1 it is launched under
``torch.distributed.run`` with one rank per GPU (RCCL over xGMI); launched directly with N>1 it
re-launches itself that way as a child process. Per-GPU batch is fixed (weak scaling); the timed
region holds exactly K full training steps — device-side input conversion, forward, loss, backward
with the bucketed all-reduce, and the fused optimizer update — bracketed by a barrier and
``torch.cuda.synchronize()``; the max over ranks is reported by rank 0 as one JSON line.
Data: synthetic (random inputs + labels resident on each GPU); weights random-init.

Other BASELINE.json configs: ``--model bert_base`` (seq 512, MultiWorkerMirroredStrategy, tokens/s),
``--model gpt2_medium_fp8`` (ctx 1024, fp8 projections, MirroredStrategy, tokens/s) and ``--model resnet50_ps``
(ParameterServerStrategy: 2 PS + 6 trainers, one task per GPU, with ``--gpus 8``; 1 PS + 3 trainers on one GPU with
``--gpus 1``; distributed_tensorflow_amd/cli/ps_bench.py).
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# Per-GPU batch, sized for the 288 GB of HBM3E (round 5; rounds 1-4 ran ResNet 256, BERT 32, GPT-2 8): per-step fixed
# costs (the optimizer pass over 110-355M parameters, embedding / loss, small layers and GEMM tile rounds that cannot
# fill 256 CUs, launch tails) are amortised over more samples. Measured on one MI355X (graph replay unless noted;
# profiles/r5_batch_sweeps.txt): ResNet-50 256 12,316-12,348 | 512 12,948-12,976 | 1024 13,188 img/s; BERT-base
# 32 878k | 64 919k | 128 1,014k tok/s; GPT-2-medium bf16 (eager) 8 238k | 16 291k | 32 309k, fp8 8 260k | 16 319k |
# 32 334k tok/s.
DEFAULT_BATCH = {"resnet50_ps": 256, "resnet50": 1024, "resnet101": 512, "resnet152": 512, "bert_base": 128, "gpt2_medium_fp8": 32,
                 "gpt2_medium": 32}
# hipGraph replay (graphs.py per-stream capture) vs eager, interleaved on one MI355X (profiles/r5_hipgraph_default.txt):
# ResNet-50 +1.4%, BERT-base +0.7%, GPT-2-medium fp8 +0.3..2%; GPT-2-medium bf16 -1.8% at batch 8 (its many
# side->main joins are device-flag waits in the replay), -0.3% at the default batch 32. Multi-rank runs are captured
# the same way when the gradient buckets go through the framework's RCCL communicator (the default): the bucket
# all-reduces are nodes of the communication stream's graph (keras Model.make_train_function; DTF_GRAPH_DIST=0 keeps
# them eager).
GRAPH_DEFAULT = {"resnet50": 1, "resnet101": 1, "resnet152": 1, "bert_base": 1, "gpt2_medium_fp8": 1, "gpt2_medium": 1}


def _relaunch(args):
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def build(args, strategy, dev, rank):
    import torch
    from distributed_tensorflow_amd.data import synthetic_imagenet, synthetic_tokens
    from distributed_tensorflow_amd.keras import losses, optimizers
    m = args.model
    with strategy.scope():
        if m.startswith("resnet"):
            from distributed_tensorflow_amd.models import ResNet
            model = ResNet(int(m[6:]), num_classes=1000)
            model.compile(optimizer=optimizers.SGD(args.lr, momentum=0.9),
                          loss=losses.SparseCategoricalCrossentropy(from_logits=True))
            data = iter(synthetic_imagenet(args.batch, dev, seed=1234 + rank))
            return model, data, "images/sec", {"model": f"ResNet-{m[6:]} v1.5", "image_size": 224, "seq_len": None}
        if m == "bert_base":
            from distributed_tensorflow_amd.models.transformer import BertModel
            model = BertModel()
            model.compile(optimizer=optimizers.AdamW(1e-4, weight_decay=0.01, epsilon=1e-6),
                          loss=losses.SparseCategoricalCrossentropy(from_logits=True))
            S, P = 512, 76
            g = torch.Generator().manual_seed(rank)
            ids = torch.randint(0, 30522, (args.batch, S), generator=g).to(dev)
            mpos = torch.stack([torch.randperm(S, generator=g)[:P] for _ in range(args.batch)]).to(dev)
            lab = torch.randint(0, 30522, (args.batch, P), generator=g).to(dev)
            x = {"input_ids": ids, "masked_positions": mpos, "token_type_ids": torch.zeros_like(ids),
                 "attention_mask": torch.ones(args.batch, S, device=dev)}

            def gen():
                while True:
                    yield x, lab
            args.tokens_per_sample = S
            return model, gen(), "tokens/sec", {"model": "BERT-base (MLM, 76 masked/seq)", "seq_len": S}
        if m.startswith("gpt2_medium"):
            from distributed_tensorflow_amd.models.transformer import gpt2_medium
            model = gpt2_medium(fp8=m.endswith("fp8"))
            model.compile(optimizer=optimizers.AdamW(3e-4, weight_decay=0.1),
                          loss=losses.SparseCategoricalCrossentropy(from_logits=True))
            S = 1024
            args.tokens_per_sample = S
            data = iter(synthetic_tokens(args.batch, S, 50257, dev, seed=rank))
            return model, data, "tokens/sec", {"model": "GPT-2-medium" + (" fp8 (e4m3 x e4m3 fwd, e5m2 x e4m3 bwd projections)" if
                                                                           m.endswith("fp8") else ""), "seq_len": S}
    raise ValueError(m)


def main():
    if os.environ.get("DTF_BENCH_WATCHDOG"):  # debugging: dump every thread's stack (and exit) after N seconds
        import faulthandler
        faulthandler.dump_traceback_later(float(os.environ["DTF_BENCH_WATCHDOG"]), exit=True)
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=None, help="per-GPU batch")
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--lr", type=float, default=0.1)
    ap.add_argument("--bucket-mb", type=float, default=None)
    ap.add_argument("--allreduce-dtype", default=None, choices=["f32", "bf16"],
                    help="gradient all-reduce payload type (default f32; bf16 halves the xGMI bytes)")
    ap.add_argument("--zero", type=int, default=0,
                    help="1: ZeRO-1 sharded optimizer update (reduce-scatter + 1/N update + all-gather of masters)")
    ap.add_argument("--graph", type=int, default=None,
                    help="1: capture the train step as per-stream hipGraphs (compile(jit_compile=True)), 0: eager; "
                         "default: per model from the interleaved A/B (profiles/r5_hipgraph_default.txt)")
    ap.add_argument("--ar-sweep", type=int, default=1,
                    help="N>1: after the timed steps, time f32 all-reduces of 1-128 MB and report RCCL bus bandwidth")
    ap.add_argument("--hiprio", type=int, default=None,
                    help="1: issue the train step on a high-priority HIP stream (the weight-gradient side stream keeps "
                         "normal priority, so the dgrad critical path wins block dispatch whenever a CU frees up); "
                         "single replica, interleaved on one MI355X: ResNet-50 13,386 / 13,459 vs 13,317 / 13,337 "
                         "img/s, GPT-2 +0.3%%, BERT +-0 (profiles/r5_hipgraph_default.txt). Default: 1 for a single "
                         "replica, 0 on the collective path, where the high-priority main stream costs 11%% "
                         "(forced-collective ResNet-50: 11,943 vs 13,436 img/s, profiles/r6_forced_collective.txt)")
    ap.add_argument("--ps", type=int, default=None, help="resnet50_ps: parameter-server tasks (default: see ps_bench)")
    ap.add_argument("--trainers", type=int, default=None, help="resnet50_ps: trainer tasks")
    ap.add_argument("--ps-cpu", action="store_true", help="resnet50_ps: PS shards in host shared memory")
    ap.add_argument("--ps-timeout", type=float, default=1500, help="resnet50_ps: whole-cluster time limit (s)")
    args = ap.parse_args()
    if args.batch is None:
        args.batch = DEFAULT_BATCH[args.model]
    if args.model.endswith("_ps"):  # its own launcher (one task per GPU), never torchrun's
        from distributed_tensorflow_amd.cli import ps_bench
        return ps_bench.main(args, sys.argv[1:])
    if args.graph is None:
        # the capture is the third call of the step (two eager warmups first): with fewer than 3 warmup steps it
        # would land in the timed region, so the default is eager then
        args.graph = GRAPH_DEFAULT.get(args.model, 0) if args.warmup >= 3 else 0
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus > 1 and world == 1 and "RANK" not in os.environ:
        return _relaunch(args)  # before anything touches the GPU
    if args.hiprio is None:  # (see --hiprio: a win for one replica, a loss with the collectives)
        args.hiprio = int(world == 1 and os.environ.get("DTF_FORCE_COLLECTIVE", "0") != "1")

    import torch
    import torch.distributed as dist

    from distributed_tensorflow_amd import parallel

    co = parallel.CommunicationOptions(wire_dtype=args.allreduce_dtype)
    if args.model == "bert_base":
        strategy = parallel.MultiWorkerMirroredStrategy(communication_options=co, bucket_mb=args.bucket_mb,
                                                        shard_optimizer=bool(args.zero))
    else:
        strategy = parallel.MirroredStrategy(bucket_mb=args.bucket_mb, communication_options=co,
                                             shard_optimizer=bool(args.zero))
    rank = strategy.worker_index
    dev = strategy.device
    if args.hiprio:
        hs = torch.cuda.Stream(device=dev, priority=-1)
        hs.wait_stream(torch.cuda.current_stream(dev))
        torch.cuda.set_stream(hs)
    model, data, unit, cfg = build(args, strategy, dev, rank)
    model._jit = bool(args.graph)
    train_fn = model.make_train_function(force=True)
    cfg["hiprio"] = bool(args.hiprio)

    def step():
        x, y = next(data)
        return train_fn((x, y))

    for _ in range(args.warmup):
        logs = step()
    cfg["hipgraph"] = bool(getattr(train_fn, "captured", False))
    sc = getattr(train_fn, "sc", None)
    if sc is not None:  # the per-stream capture: graphs (streams) and cross-stream edges by kind
        cfg["graph_streams"] = len(sc.streams)
        cfg["graph_edges"] = dict(sc.counts)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    bucketers = list(getattr(strategy, "_bucketers", {}).values())
    for b in bucketers:
        b.timing = hasattr(b, "exposed_ms")
    t0 = time.perf_counter()
    for _ in range(args.steps):
        logs = step()
    t_issue = time.perf_counter() - t0  # host time to issue the K steps (the GPU may still be running)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if hasattr(train_fn, "check"):
        train_fn.check()  # a timed-out cross-stream wait of the graph replay fails the run (not a slow or wrong one)
    exposed = [b.exposed_ms() for b in bucketers if hasattr(b, "exposed_ms")]
    exposed = [e for e in exposed if e is not None]
    # the loss and the replica checksum describe exactly the warmup + timed steps (taken before the probe below)
    loss = float(logs["loss"])
    # proof that the N replicas trained in lock step: an exact checksum of every trainable f32 master (the bit
    # patterns summed as integers), compared across ranks (min == max); the world size the process group reports
    arena = getattr(model, "_arena", None)
    csum = int(arena.flat.detach().view(torch.int32).to(torch.int64).sum().item()) if arena is not None else 0
    # after the timed region: the host time to issue ONE step into an idle GPU queue (min of 3). In the timed loop
    # the host is throttled by the queue once it runs ahead, so its issue time there equals the GPU time either way;
    # this one says whether Python + launches alone would keep up with the GPU. (These 3 extra steps change the
    # weights after the loss / checksum above were taken.)
    single = []
    for _ in range(3):
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        step()
        single.append(time.perf_counter() - t1)
    torch.cuda.synchronize()
    rccl_world = dist.get_world_size() if dist.is_initialized() else 1
    backend = dist.get_backend() if dist.is_initialized() else None
    identical = True
    if dist.is_initialized():
        mm = torch.tensor([csum, -csum], dtype=torch.int64, device=dev)
        dist.all_reduce(mm, op=dist.ReduceOp.MAX)
        identical = int(mm[0].item()) == csum and int(-mm[1].item()) == csum
    t = torch.tensor([dt, sum(exposed) if exposed else 0.0], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)  # slowest rank's clock and exposed communication
    dt, exposed_max = float(t[0].item()), float(t[1].item())
    # after the timed region (it changes nothing that was measured): the collective's own bus bandwidth on this
    # node at bucket-sized messages, so the bucket cap and wire dtype can be chosen from a measurement on the
    # hardware the scaling run used (RCCL over xGMI on an 8-GPU node)
    ar_sweep = _allreduce_sweep(dist, dev, world, bucketers) if (world > 1 and args.ar_sweep) else None
    ms = dt / args.steps * 1e3
    global_batch = args.batch * world
    per_sample = getattr(args, "tokens_per_sample", 1)
    value = global_batch * per_sample * args.steps / dt
    if rank == 0:
        with open(os.path.join(ROOT, "BASELINE.json")) as f:
            base = json.load(f)
        pub = base.get("published") or {}
        ref = pub.get(args.model) if isinstance(pub, dict) else None
        metric = base["metric"] if args.model == "resnet50" else f"{unit} (whole node) {cfg['model']}"
        out = {
            "metric": metric,
            "value": round(value, 2),
            "unit": unit,
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": (value / ref) if ref else None,
            "dtype": "bf16+fp8" if args.model.endswith("fp8") else "bf16",
            "data": "synthetic (random inputs + labels resident on GPU; random-init weights)",
            "config": dict(cfg, global_batch=global_batch, per_gpu_batch=args.batch, parallelism=f"dp{world}",
                           strategy=type(strategy).__name__ + " (1 process/GPU, %s)" % (
                               ("RCCL" if dist.get_backend() == "nccl" else dist.get_backend())
                               if dist.is_initialized() else "single replica"),
                           optimizer=type(model.optimizer).__name__, final_loss=round(loss, 4),
                           allreduce_dtype=args.allreduce_dtype or "f32", zero1=bool(args.zero),
                           bucket_mb=getattr(bucketers[0], "bucket_mb", None) if bucketers else None,
                           exposed_comm_ms_per_step=round(exposed_max, 3),
                           # bucket collectives issued (warmup + timed steps) per path: RCCL, or the one-shot P2P
                           # all-reduce over IPC-mapped peer arenas for buckets <= DTF_P2P_MAX_KB (parallel/p2p.py)
                           allreduce_paths=_paths(bucketers),
                           forced_collective=os.environ.get("DTF_FORCE_COLLECTIVE", "0") == "1"),
            # host time spent issuing a step (Python + launches); close to ms_per_step = the host, not the GPU, paces
            # the run (what hipGraph capture, bench.py --graph 1, removes)
            "host_issue_ms_per_step": round(t_issue / args.steps * 1e3, 3),
            "host_issue_ms_single_step": round(min(single) * 1e3, 3),
            "rccl_world": rccl_world,
            "allreduce_busbw_GBps": ar_sweep,
            "process_group_backend": backend,
            "replicas_identical": identical,
            "weights_checksum": csum,
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return 0


def _paths(bucketers):
    out = {}
    for b in bucketers:
        for k, v in (getattr(b, "paths", None) or {}).items():
            out[k] = out.get(k, 0) + v
    return out or None


def _allreduce_sweep(dist, dev, world, bucketers, sizes_mb=(1, 4, 16, 32, 64, 128), iters=5,
                     min_channels=(4, 8, 16)):
    """Bus bandwidth (GB/s, the nccl-tests convention: bytes * 2 (n-1) / n / time) of f32 all-reduces, slowest rank's
    time per size, on the communicator the gradient buckets actually use — the framework's RCCL communicator
    (parallel/rccl.py) at the bucketer's channel setting — plus the same communicator type at min_channels 4 / 8 / 16
    (the bucket cap and channel count are chosen from this table) and torch's ProcessGroupNCCL for comparison."""
    import torch
    from distributed_tensorflow_amd.parallel import rccl
    sync = torch.cuda.synchronize if dev.type == "cuda" else (lambda: None)

    def sweep(fn):
        out = {}
        for mb in sizes_mb:
            x = torch.ones(mb * (1 << 20) // 4, dtype=torch.float32, device=dev)
            for _ in range(2):
                fn(x)
            sync()
            dist.barrier()
            t0 = time.perf_counter()
            for _ in range(iters):
                fn(x)
            sync()
            el = torch.tensor([(time.perf_counter() - t0) / iters], dtype=torch.float64, device=dev)
            dist.all_reduce(el, op=dist.ReduceOp.MAX)
            out[f"{mb}MB"] = round(mb * (1 << 20) * 2 * (world - 1) / world / float(el.item()) / 1e9, 1)
            del x
        return out

    res = {}
    used = next((b.rccl for b in bucketers if getattr(b, "rccl", None) is not None), None)
    if used is not None:
        res["buckets"] = {"communicator": "native", "min_channels": used.min_channels,
                          "max_channels": used.max_channels, "busbw": sweep(used.all_reduce_)}
    if dev.type == "cuda" and dist.get_backend() == "nccl" and rccl.available()[0]:
        for mc in min_channels:
            c = rccl.RcclCommunicator(device=dev, min_channels=mc, max_channels=max(mc, rccl.DEFAULT_MAX_CHANNELS),
                                      name=f"sweep{mc}")
            try:
                res[f"native_min{mc}"] = sweep(c.all_reduce_)
            finally:
                c.destroy()
    res["torch_process_group"] = sweep(lambda x: dist.all_reduce(x))
    return res


if __name__ == "__main__":
    sys.exit(main())
