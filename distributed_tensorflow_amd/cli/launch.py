"""Local cluster launcher: the reference runbook (README.md:9-27) as one command.

    python -m distributed_tensorflow_amd.cli.launch --ps 1 --workers 1 --chief 1 \
        [--gpus 0,1,...] -- python -m distributed_tensorflow_amd.cli.train --optimizer=adam

Every task gets its own process, a free 127.0.0.1 port and a ``TF_CONFIG`` naming the whole
cluster (chief job ``master``, like the reference). With ``--gpus`` the chief/worker tasks get
one GPU each through ``DTF_DEVICE_ORDINAL`` (PS tasks too when ``--ps_gpus``), an index into the launcher's own
visible devices (its ``HIP_VISIBLE_DEVICES`` is inherited unchanged), all of them staying visible so
the tasks can map each other's HBM (the PS data plane, parallel/ps_shm.py), otherwise
``HIP_VISIBLE_DEVICES=''`` (the README runs everything on CPU). Exit code: the first non-zero
task exit code, else 0. Output lines are prefixed with the task name.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import threading


def free_ports(n):
    socks, ports = [], []
    for _ in range(n):
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        socks.append(s)
        ports.append(s.getsockname()[1])
    for s in socks:
        s.close()
    return ports


def make_cluster(num_ps, num_workers, num_chief, chief_job="master"):
    ports = free_ports(num_ps + num_workers + num_chief)
    it = iter(ports)
    cluster = {}
    if num_ps:
        cluster["ps"] = [f"127.0.0.1:{next(it)}" for _ in range(num_ps)]
    if num_workers:
        cluster["worker"] = [f"127.0.0.1:{next(it)}" for _ in range(num_workers)]
    if num_chief:
        cluster[chief_job] = [f"127.0.0.1:{next(it)}" for _ in range(num_chief)]
    return cluster


def _pump(prefix, stream, out):
    for line in iter(stream.readline, b""):
        out.write(f"[{prefix}] {line.decode(errors='replace')}")
        out.flush()


def task_list(num_ps, num_workers, num_chief, chief_job="master"):
    """Launch order of the tasks: PS tasks, then the chief, then the workers."""
    return [("ps", i) for i in range(num_ps)] + [(chief_job, i) for i in range(num_chief)] + \
        [("worker", i) for i in range(num_workers)]


def assign_devices(tasks, gpu_list, ps_gpus=False):
    """{task: device ordinal string}: the GPU tasks (chief/worker, and PS when ps_gpus) take `gpu_list` round-robin in
    launch order; a task not in the result runs on the host (HIP_VISIBLE_DEVICES='')."""
    out = {}
    gi = 0
    for t, i in tasks:
        if gpu_list and (t != "ps" or ps_gpus):
            out[(t, i)] = gpu_list[gi % len(gpu_list)]
            gi += 1
    return out


def launch(cmd, num_ps=1, num_workers=1, num_chief=1, gpus=None, ps_gpus=False, chief_job="master", env=None,
           timeout=None, log=sys.stdout, host_kv=False, max_restarts=0):
    """Start every task and supervise them.

    host_kv: the launcher itself hosts the coordination KV store (DTF_KV_ADDR), so it outlives any task.
    max_restarts: a chief/worker task that exits abnormally is restarted (same TF_CONFIG and port, without
    DTF_FAULT) up to this many times in total — the "kill -9 the chief, relaunch, restore from the
    checkpoint" recovery path. Requires host_kv (the chief would otherwise take the
    coordination service down with it)."""
    import time
    cluster = make_cluster(num_ps, num_workers, num_chief, chief_job)
    tasks = task_list(num_ps, num_workers, num_chief, chief_job)
    gpu_list = [g for g in (gpus.split(",") if gpus else []) if g != ""]
    ordinals = assign_devices(tasks, gpu_list, ps_gpus)
    kv_server = None
    if host_kv or max_restarts:
        from ..parallel.kv import KVServer
        kv_server = KVServer("127.0.0.1", 0)
    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    envs = {}
    for t, i in tasks:
        e = dict(os.environ, **(env or {}))
        e["PYTHONPATH"] = root + (os.pathsep + e["PYTHONPATH"] if e.get("PYTHONPATH") else "")
        e["TF_CONFIG"] = json.dumps({"cluster": cluster, "task": {"type": t, "index": i}})
        e["DTF_ROLE"] = f"{t}{i}"
        if kv_server is not None:
            e["DTF_KV_ADDR"] = f"127.0.0.1:{kv_server.port}"
        if (t, i) in ordinals:
            # every GPU of the launcher's own visible set stays visible (a PS shard in one GPU's HBM is mapped by
            # the trainers on the others); the task's device is selected by its ordinal WITHIN that set, so
            # --gpus indexes the caller's HIP_VISIBLE_DEVICES (left untouched), never raw physical ids
            e["DTF_DEVICE_ORDINAL"] = ordinals[(t, i)]
        else:
            e["HIP_VISIBLE_DEVICES"] = ""
            e["CUDA_VISIBLE_DEVICES"] = ""
        envs[(t, i)] = e

    def spawn(t, i, e):
        p = subprocess.Popen(cmd, env=e, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
        th = threading.Thread(target=_pump, args=(f"{t}{i}", p.stdout, log), daemon=True)
        th.start()
        return p, th

    procs = {(t, i): spawn(t, i, envs[(t, i)]) for t, i in tasks}
    restarts = 0
    rc = 0
    deadline = None if timeout is None else time.time() + timeout
    try:
        running = set(procs)
        while running:
            for key in list(running):
                p, th = procs[key]
                r = p.poll()
                if r is None:
                    continue
                th.join(timeout=5)
                t, i = key
                if r != 0 and t != "ps" and restarts < max_restarts:
                    restarts += 1
                    log.write(f"[launch] {t}{i} exited with {r}; restart {restarts}/{max_restarts}\n")
                    log.flush()
                    e = dict(envs[key])
                    e.pop("DTF_FAULT", None)
                    e["DTF_RESTART"] = str(restarts)
                    procs[key] = spawn(t, i, e)
                    continue
                running.discard(key)
                if r != 0 and rc == 0:
                    rc = r
            if deadline is not None and time.time() > deadline:
                rc = 124
                break
            time.sleep(0.05)
    finally:
        for p, th in procs.values():
            if p.poll() is None:
                p.kill()
        if kv_server is not None:
            kv_server.stop()
    return rc, cluster


def main(argv=None):
    ap = argparse.ArgumentParser("dtf-launch")
    ap.add_argument("--ps", type=int, default=1)
    ap.add_argument("--workers", type=int, default=1)
    ap.add_argument("--chief", type=int, default=1)
    ap.add_argument("--chief_job", default="master")
    ap.add_argument("--gpus", default=None)
    ap.add_argument("--ps_gpus", action="store_true")
    ap.add_argument("--timeout", type=float, default=None)
    ap.add_argument("--host_kv", action="store_true", help="launcher hosts the coordination KV store")
    ap.add_argument("--max_restarts", type=int, default=0, help="restart failed chief/worker tasks")
    ap.add_argument("cmd", nargs=argparse.REMAINDER)
    a = ap.parse_args(argv)
    cmd = a.cmd[1:] if a.cmd and a.cmd[0] == "--" else a.cmd
    if not cmd:
        cmd = [sys.executable, "-m", "distributed_tensorflow_amd.cli.train"]
    rc, _ = launch(cmd, a.ps, a.workers, a.chief, a.gpus, a.ps_gpus, a.chief_job, timeout=a.timeout,
                   host_kv=a.host_kv, max_restarts=a.max_restarts)
    return rc


if __name__ == "__main__":
    sys.exit(main())
