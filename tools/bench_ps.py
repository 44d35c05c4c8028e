#!/usr/bin/env python
"""BASELINE.json config #4: ResNet-50 under ParameterServerStrategy (2 PS + 6 trainers on one 8-GPU node).

    python tools/bench_ps.py --gpus 8 [--steps 20 --warmup 5 --batch 256]

Without TF_CONFIG it launches the local cluster itself (cli.launch: one process per task, every GPU visible, the
task's own GPU by ordinal, launcher-hosted coordination store): `--ps` parameter servers (default
max(1, gpus // 4)) holding the variable shards in their HBM, `--trainers` trainers (default the remaining GPUs; the
first is the chief). Tasks are assigned GPUs round-robin over `--gpus`, so `--gpus 1 --ps 1 --trainers 3` rehearses
the whole data plane on one GPU. The data plane is the one the chief negotiates — on one node `shm`: gradients are
copied into per-trainer inboxes in the PS's HBM (HIP IPC, xGMI between GPUs) and parameters copied back out, a
shared-memory mailbox carries the requests (parallel/ps_shm.py); `--ps_cpu` keeps the shards in host shared memory.
Training is asynchronous as in the reference: every trainer pushes its gradients to the PS shards after each step
and continues with the values it pulls.
After `--warmup` steps every trainer waits at a coordination-store barrier, then runs `--steps` steps; each reports
its wall-clock (start, end) window and the chief prints one JSON line whose value is ALL images processed divided by
(latest end - earliest start): a whole-node throughput over one common window (summing per-trainer
rates over non-coincident windows overstated it). With at least as many GPUs as tasks it also checks that every
task sits on its own GPU and that the trainers reach the PS shards through the HIP-IPC peer path.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=8)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--depth", type=int, default=50)
    ap.add_argument("--ps", type=int, default=None, help="PS tasks (default max(1, gpus // 4))")
    ap.add_argument("--trainers", type=int, default=None, help="trainer tasks (default: the remaining GPUs)")
    ap.add_argument("--ps_cpu", action="store_true", help="PS shards in host shared memory")
    ap.add_argument("--timeout", type=float, default=1500)
    return ap.parse_args()


def launch(a):
    from distributed_tensorflow_amd.cli.launch import launch as run_cluster
    n_ps = a.ps if a.ps is not None else (1 if a.ps_cpu else max(1, a.gpus // 4))
    n_tr = a.trainers if a.trainers is not None else (a.gpus if a.ps_cpu else a.gpus - n_ps)
    if n_tr < 1:
        raise SystemExit("need at least one trainer (pass --trainers on a 1-GPU box)")
    env = {"DTF_BENCH_PS_CPU": "1" if a.ps_cpu else "0"}
    cmd = [sys.executable, os.path.abspath(__file__)] + sys.argv[1:]
    gpus = ",".join(str(i) for i in range(a.gpus))  # PS tasks first, then trainers, round-robin
    rc, _ = run_cluster(cmd, num_ps=n_ps, num_workers=n_tr - 1, num_chief=1, gpus=gpus, ps_gpus=not a.ps_cpu,
                        env=env, timeout=a.timeout, host_kv=True)
    return rc


def task(a):
    import torch
    from distributed_tensorflow_amd.parallel import TFConfigClusterResolver
    from distributed_tensorflow_amd.parallel.parameter_server import ParameterServerStrategy, run_parameter_server
    r = TFConfigClusterResolver()
    ps_cpu = os.environ.get("DTF_BENCH_PS_CPU") == "1"
    from distributed_tensorflow_amd import context
    if r.is_ps:
        return run_parameter_server(r, device="cpu" if ps_cpu else context.default_device())
    from distributed_tensorflow_amd.data import synthetic_imagenet
    from distributed_tensorflow_amd.keras import losses, optimizers
    from distributed_tensorflow_amd.models import ResNet
    dev = context.default_device()
    strat = ParameterServerStrategy(r, variable_partitioner="balanced", device=dev)
    with strat.scope():
        model = ResNet(a.depth, num_classes=1000)
        model.compile(optimizer=optimizers.SGD(0.1, momentum=0.9),
                      loss=losses.SparseCategoricalCrossentropy(from_logits=True))
    data = iter(synthetic_imagenet(a.batch, dev, seed=1234 + strat.worker_index))
    for _ in range(a.warmup):
        logs = model.train_step(next(data))
    torch.cuda.synchronize()
    # every trainer starts its timed window together (coordination-store barrier)
    strat.kv.add("bench/ready", 1)
    strat.kv.wait_ge("bench/ready", strat.num_workers, timeout_s=600)
    t0 = time.time()
    for _ in range(a.steps):
        logs = model.train_step(next(data))
    torch.cuda.synchronize()
    t1 = time.time()
    ips = a.batch * a.steps / (t1 - t0)
    peer = bool(strat._shm is not None and any(r_.desc.get("kind") == "hip" for r_ in strat._shm.inbox))
    strat.kv.set(f"bench/{strat.worker_index}", json.dumps({"ips": ips, "ms": (t1 - t0) / a.steps * 1e3,
                                                            "t0": t0, "t1": t1, "loss": float(logs["loss"]),
                                                            "ipc_peer": peer}))
    if strat.is_chief:
        res = [json.loads(strat.kv.get(f"bench/{i}").decode()) for i in range(strat.num_workers)]
        span = max(x["t1"] for x in res) - min(x["t0"] for x in res)
        total = a.batch * a.steps * len(res) / span
        roles = [f"ps{i}" for i in range(r.cluster.num_tasks("ps"))] + [f"{t}{i}" for t, i in r.trainer_tasks()]
        devs = {ro: json.loads(strat.kv.get(f"task/{ro}/dev").decode())["device"] for ro in roles}
        own_gpu = len(set(devs.values())) == len(devs) and all(d.startswith("cuda") for d in devs.values())
        if a.gpus >= len(roles) and not ps_cpu:
            # the 8-GPU layout must really be one task per GPU over the IPC peer path
            assert own_gpu, f"tasks share GPUs: {devs}"
            assert strat.transport == "shm" and all(x["ipc_peer"] for x in res), "PS data plane is not HIP IPC"
        print(json.dumps({
            "metric": f"images/sec (whole node) ResNet-{a.depth} bf16, ParameterServerStrategy (async)",
            "value": round(total, 2), "unit": "images/sec", "n_gpus": a.gpus, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": round(max(x["ms"] for x in res), 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "bf16", "data": "synthetic",
            "config": {"model": f"ResNet-{a.depth} v1.5", "per_trainer_batch": a.batch,
                       "ps_tasks": r.cluster.num_tasks("ps"), "trainers": strat.num_workers,
                       "ps_device": "cpu" if ps_cpu else "gpu", "transport": strat.transport,
                       "staleness": strat.staleness, "overlap_push": strat.overlap_push,
                       "task_devices": devs, "one_task_per_gpu": own_gpu,
                       "ipc_peer_path": all(x["ipc_peer"] for x in res),
                       "aggregate": "all images / (latest end - earliest start) after a store barrier",
                       "window_s": round(span, 3),
                       "per_trainer_images_per_sec": [round(x["ips"], 1) for x in res]}}), flush=True)
    strat.shutdown()
    return 0


def main():
    a = parse()
    if not os.environ.get("TF_CONFIG"):
        return launch(a)
    return task(a)


if __name__ == "__main__":
    sys.exit(main())
