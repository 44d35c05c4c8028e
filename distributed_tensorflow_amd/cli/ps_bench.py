"""BASELINE.json config #4: ResNet-50 under ParameterServerStrategy, 2 PS + 6 trainers on one 8-GPU node.

Entry point: ``python bench.py --model resnet50_ps --gpus N [--steps K --warmup W --batch B]`` (the driver's bench
contract). Without TF_CONFIG the call launches the local cluster itself (cli.launch: one process per task, every GPU
visible, each task bound to its own GPU by ordinal, launcher-hosted coordination store) and re-runs the same command
line in every task:

* ``--gpus 8``: 2 parameter servers holding the variable shards in their HBM + 6 trainers (the first is the chief),
  one task per GPU (``plan``); the chief asserts that layout and that trainers reach the shards over the HIP-IPC
  peer path (xGMI between GPUs);
* ``--gpus 1``: 1 PS + 3 trainers sharing cuda:0 — the whole data plane rehearsed on one GPU;
* other N: max(1, N // 4) PS tasks and the remaining GPUs as trainers.

Training is asynchronous as in the reference (/root/reference/trainer/task.py:117-127, 232-236): every trainer pushes
its gradients to the PS shards after each step and continues with the values it pulls; the PS applies the fused
optimizer to its shards. After ``--warmup`` steps every trainer waits at a coordination-store barrier, then runs
``--steps`` steps and reports its wall-clock window; the chief prints ONE JSON line (unprefixed, on the launcher's
stdout) whose value is ALL images processed divided by (latest end - earliest start). PS tasks exit once every
trainer is done (/root/reference/auto_stop_ps/task.py:127-150).
"""
from __future__ import annotations

import io
import json
import os
import sys
import time


def plan(gpus, ps=None, trainers=None, ps_cpu=False):
    """(PS tasks, trainer tasks) for a node of `gpus` GPUs (see the module docstring)."""
    n_ps = ps if ps is not None else (1 if ps_cpu or gpus < 4 else max(1, gpus // 4))
    if trainers is not None:
        n_tr = trainers
    elif ps_cpu:
        n_tr = gpus
    elif gpus == 1:
        n_tr = 3
    else:
        n_tr = gpus - n_ps
    if n_tr < 1:
        raise SystemExit("parameter-server bench: need at least one trainer (pass --trainers)")
    return n_ps, n_tr


def layout(gpus, n_ps, n_tr, ps_cpu=False):
    """{role: device ordinal} exactly as cli.launch assigns it (PS first, then the chief, then the workers)."""
    from .launch import assign_devices, task_list
    tasks = task_list(n_ps, n_tr - 1, 1)
    devs = assign_devices(tasks, [str(i) for i in range(gpus)], ps_gpus=not ps_cpu)
    return {f"{t}{i}": devs.get((t, i)) for t, i in tasks}


class _Tee(io.TextIOBase):
    """Launcher log sink: the chief's JSON result line goes to stdout without its task prefix, everything else to
    stderr (the driver reads ONE JSON line from stdout)."""

    def __init__(self):
        self.result = None

    def write(self, s):
        for line in s.splitlines(True):
            body = line.split("] ", 1)[1] if line.startswith("[") and "] " in line else line
            if body.startswith("{\"metric\"") and line.startswith("[master0]"):
                self.result = body.strip()
                sys.stdout.write(body)
                sys.stdout.flush()
            else:
                sys.stderr.write(line)
        return len(s)

    def flush(self):
        sys.stderr.flush()


def launch(args, argv):
    from .launch import launch as run_cluster
    n_ps, n_tr = plan(args.gpus, args.ps, args.trainers, args.ps_cpu)
    env = {"DTF_BENCH_PS_CPU": "1" if args.ps_cpu else "0", "DTF_BENCH_PS_GPUS": str(args.gpus)}
    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    cmd = [sys.executable, os.path.join(root, "bench.py")] + list(argv)
    gpus = ",".join(str(i) for i in range(args.gpus))
    tee = _Tee()
    rc, _ = run_cluster(cmd, num_ps=n_ps, num_workers=n_tr - 1, num_chief=1, gpus=gpus, ps_gpus=not args.ps_cpu,
                        env=env, timeout=args.ps_timeout, host_kv=True, log=tee)
    if rc == 0 and tee.result is None:
        sys.stderr.write("parameter-server bench: the chief printed no result\n")
        return 1
    return rc


def task(args):
    import torch
    from .. import context
    from ..data import synthetic_imagenet
    from ..keras import losses, optimizers
    from ..models import ResNet
    from ..parallel import TFConfigClusterResolver
    from ..parallel.parameter_server import ParameterServerStrategy, run_parameter_server
    r = TFConfigClusterResolver()
    ps_cpu = os.environ.get("DTF_BENCH_PS_CPU") == "1"
    gpus = int(os.environ.get("DTF_BENCH_PS_GPUS", args.gpus))
    if r.is_ps:
        return run_parameter_server(r, device="cpu" if ps_cpu else context.default_device())
    depth = int(args.model[len("resnet"):].split("_")[0])
    dev = context.default_device()
    strat = ParameterServerStrategy(r, variable_partitioner="balanced", device=dev)
    with strat.scope():
        model = ResNet(depth, num_classes=1000)
        model.compile(optimizer=optimizers.SGD(args.lr, momentum=0.9),
                      loss=losses.SparseCategoricalCrossentropy(from_logits=True))
    data = iter(synthetic_imagenet(args.batch, dev, seed=1234 + strat.worker_index))
    sync = torch.cuda.synchronize if dev.type == "cuda" else (lambda: None)
    for _ in range(args.warmup):
        logs = model.train_step(next(data))
    sync()
    # every trainer starts its timed window together (coordination-store barrier)
    strat.kv.add("bench/ready", 1)
    strat.kv.wait_ge("bench/ready", strat.num_workers, timeout_s=600)
    t0 = time.time()
    for _ in range(args.steps):
        logs = model.train_step(next(data))
    sync()
    t1 = time.time()
    ips = args.batch * args.steps / (t1 - t0)
    peer = bool(strat._shm is not None and any(r_.desc.get("kind") == "hip" for r_ in strat._shm.inbox))
    strat.kv.set(f"bench/{strat.worker_index}", json.dumps({"ips": ips, "ms": (t1 - t0) / args.steps * 1e3,
                                                            "t0": t0, "t1": t1, "loss": float(logs["loss"]),
                                                            "ipc_peer": peer}))
    if strat.is_chief:
        res = [json.loads(strat.kv.get(f"bench/{i}").decode()) for i in range(strat.num_workers)]
        span = max(x["t1"] for x in res) - min(x["t0"] for x in res)
        total = args.batch * args.steps * len(res) / span
        roles = [f"ps{i}" for i in range(r.cluster.num_tasks("ps"))] + [f"{t}{i}" for t, i in r.trainer_tasks()]
        devs = {ro: json.loads(strat.kv.get(f"task/{ro}/dev").decode())["device"] for ro in roles}
        own_gpu = len(set(devs.values())) == len(devs) and all(d.startswith("cuda") for d in devs.values())
        if gpus >= len(roles) and not ps_cpu:
            # the 8-GPU layout must really be one task per GPU over the IPC peer path
            assert own_gpu, f"tasks share GPUs: {devs}"
            assert strat.transport == "shm" and all(x["ipc_peer"] for x in res), "PS data plane is not HIP IPC"
        n_ps = r.cluster.num_tasks("ps")
        print(json.dumps({
            "metric": f"images/sec (whole node) ResNet-{depth} bf16, ParameterServerStrategy (async)",
            "value": round(total, 2), "unit": "images/sec", "n_gpus": gpus, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(max(x["ms"] for x in res), 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "bf16",
            "data": "synthetic (random inputs + labels resident on GPU; random-init weights)",
            "config": {"model": f"ResNet-{depth} v1.5", "global_batch": args.batch * strat.num_workers,
                       "per_trainer_batch": args.batch, "seq_len": None,
                       "parallelism": f"ps{n_ps}+async{strat.num_workers}",
                       "ps_tasks": n_ps, "trainers": strat.num_workers,
                       "ps_device": "cpu" if ps_cpu else "gpu", "transport": strat.transport,
                       "staleness": strat.staleness, "overlap_push": strat.overlap_push,
                       "task_devices": devs, "one_task_per_gpu": own_gpu,
                       "ipc_peer_path": all(x["ipc_peer"] for x in res),
                       "aggregate": "all images / (latest end - earliest start) after a store barrier",
                       "window_s": round(span, 3), "final_loss": round(float(logs["loss"]), 4),
                       "per_trainer_images_per_sec": [round(x["ips"], 1) for x in res]}}), flush=True)
    strat.shutdown()
    return 0


def main(args, argv):
    """bench.py --model resnet<depth>_ps: the launcher side without TF_CONFIG, a task of the cluster with it."""
    if os.environ.get("TF_CONFIG"):
        return task(args)
    if int(os.environ.get("RANK", "0")) != 0:
        return 0  # started under torchrun: rank 0 launches the whole cluster (one task per GPU) by itself
    return launch(args, argv)
