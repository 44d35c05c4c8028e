"""Cluster topology from TF_CONFIG (and torchrun's environment).

Reference behaviour (trainer/task.py:59,109-119; auto_stop_ps/task.py:111-125):
an empty/absent ``TF_CONFIG`` means standalone training; otherwise it is JSON
``{"cluster": {job: [host:port, ...]}, "task": {"type": ..., "index": ...}}``
with jobs ``ps``, ``worker`` and ``master`` (the chief). We accept ``chief`` as a
synonym of ``master`` and also ``evaluator``.
"""
from __future__ import annotations

import json
import os
from dataclasses import dataclass, field

CHIEF_JOBS = ("chief", "master")


@dataclass
class ClusterSpec:
    """tf.train.ClusterSpec analogue: job name -> list of "host:port"."""
    jobs: dict = field(default_factory=dict)

    def __init__(self, cluster=None):
        if isinstance(cluster, ClusterSpec):
            cluster = cluster.jobs
        self.jobs = {k: list(v) if not isinstance(v, dict) else [v[i] for i in sorted(v)]
                     for k, v in (cluster or {}).items()}

    def as_dict(self):
        return {k: list(v) for k, v in self.jobs.items()}

    @property
    def job_names(self):
        return sorted(self.jobs)

    def num_tasks(self, job):
        return len(self.jobs.get(job, []))

    def task_address(self, job, index):
        return self.jobs[job][index]

    def job_tasks(self, job):
        return list(self.jobs.get(job, []))

    def chief_job(self):
        for j in CHIEF_JOBS:
            if self.jobs.get(j):
                return j
        return None

    def __bool__(self):
        return bool(self.jobs)


class TFConfigClusterResolver:
    """Parses TF_CONFIG. Absent/empty TF_CONFIG -> standalone (reference trainer/task.py:59)."""

    def __init__(self, tf_config=None, task_type=None, task_id=None, rpc_layer="grpc"):
        raw = tf_config if tf_config is not None else os.environ.get("TF_CONFIG", "")
        if isinstance(raw, str):
            cfg = json.loads(raw) if raw.strip() else {}
        else:
            cfg = dict(raw)
        self._cfg = cfg
        self.cluster = ClusterSpec(cfg.get("cluster", {}))
        task = cfg.get("task") or {}
        self.task_type = task_type if task_type is not None else task.get("type")
        self.task_id = int(task_id if task_id is not None else task.get("index", 0) or 0)
        self.rpc_layer = cfg.get("rpc_layer", rpc_layer)
        if self.cluster and self.task_type is None:
            raise ValueError("TF_CONFIG has a cluster but no task.type")
        if self.task_type is not None and self.cluster and self.task_type not in self.cluster.jobs \
                and self.task_type != "evaluator":
            raise ValueError(f"task type {self.task_type!r} not in cluster jobs {self.cluster.job_names}")

    @property
    def standalone(self):
        return not self.cluster

    def cluster_spec(self):
        return self.cluster

    @property
    def is_chief(self):
        if self.standalone:
            return True
        chief = self.cluster.chief_job()
        if chief is None:  # no chief job: worker 0 is the chief (MWMS convention)
            return self.task_type == "worker" and self.task_id == 0
        return self.task_type in CHIEF_JOBS

    @property
    def is_ps(self):
        return self.task_type == "ps"

    def master(self):
        if self.standalone:
            return ""
        return self.cluster.task_address(self.task_type, self.task_id)

    def num_accelerators(self):
        import torch
        return {"GPU": torch.cuda.device_count()}

    def trainer_tasks(self):
        """Ordered (type, index) list of tasks that run training: chief first, then workers."""
        out = []
        c = self.cluster.chief_job()
        if c:
            out += [(c, i) for i in range(self.cluster.num_tasks(c))]
        out += [("worker", i) for i in range(self.cluster.num_tasks("worker"))]
        return out

    def trainer_rank(self):
        for r, t in enumerate(self.trainer_tasks()):
            if t == (self.task_type, self.task_id):
                return r
        return -1


class TorchrunClusterResolver:
    """RANK/WORLD_SIZE/LOCAL_RANK/MASTER_ADDR/MASTER_PORT (one process per GPU)."""

    def __init__(self):
        self.rank = int(os.environ.get("RANK", "0"))
        self.world_size = int(os.environ.get("WORLD_SIZE", "1"))
        self.local_rank = int(os.environ.get("LOCAL_RANK", "0"))
        self.master_addr = os.environ.get("MASTER_ADDR", "127.0.0.1")
        self.master_port = int(os.environ.get("MASTER_PORT", "29500"))

    @property
    def is_chief(self):
        return self.rank == 0

    @staticmethod
    def active():
        """A torchrun-style launch: several ranks, or ONE rank whose launcher also published the rendezvous address
        (torchrun --nproc-per-node 1: the worker must meet torchrun's agent store at MASTER_PORT, not a default)."""
        if "RANK" not in os.environ:
            return False
        return int(os.environ.get("WORLD_SIZE", "1")) > 1 or "MASTER_PORT" in os.environ


class SimpleClusterResolver(TFConfigClusterResolver):
    def __init__(self, cluster_spec, task_type=None, task_id=0, rpc_layer="grpc"):
        super().__init__(tf_config={"cluster": ClusterSpec(cluster_spec).as_dict(),
                                    "task": {"type": task_type, "index": task_id}})
