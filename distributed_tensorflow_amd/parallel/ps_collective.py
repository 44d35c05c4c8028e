"""Parameter-server data plane over torch.distributed point-to-point (RCCL over xGMI between GPUs; gloo on CPU).

The reference moves every parameter pull and gradient push through TF's gRPC Send/Recv rendezvous
(reference trainer/task.py:236 [TF-RT]). The TCP transport (csrc/runtime/ps_transport.cc)
keeps that shape for CPU clusters; on one MI355X node a worker pulling and pushing a ResNet-50 shard
(~100 MB each way) through host memory would spend far longer on the copy than on the step, so GPU
clusters use this transport instead:

* every ps and trainer task joins one process group (PS tasks are ranks 0..P-1, trainers P..P+T-1; the
  rendezvous address is published by ps0 through the coordination KV store);
* one 2-rank sub-group per (ps, trainer) pair, so each pair owns an RCCL communicator and a PS serves its
  trainers concurrently: one server thread per trainer, the update applied under a per-shard lock by the
  fused optimizer kernel on the PS's GPU (variables stay resident in the PS's HBM);
* a request is a small int64 header [op, n] followed by payload: PUSH (gradients, answered with the fresh
  parameters after the apply), ASSIGN (chief initialisation / restore), PULL, PULL_SLOTS, DONE. The
  trainer issues its requests to all PS shards with isend/irecv, so shards are served in parallel.
Asynchronous semantics are the reference's: every trainer applies its own gradients whenever it pushes;
there is no cross-trainer synchronisation.
"""
from __future__ import annotations

import datetime
import os
import socket
import threading

import torch
import torch.distributed as dist

OP_DONE, OP_PUSH, OP_ASSIGN, OP_PULL, OP_SLOTS = 0, 1, 2, 3, 4


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class PSGroup:
    """Process group of a PS cluster + the (ps, trainer) pair sub-groups."""

    def __init__(self, kv, resolver, device, timeout_s=900):
        self.num_ps = resolver.cluster.num_tasks("ps")
        self.num_trainers = len(resolver.trainer_tasks())
        self.world = self.num_ps + self.num_trainers
        self.rank = resolver.task_id if resolver.is_ps else self.num_ps + resolver.trainer_rank()
        self.device = device
        if self.rank == 0:  # ps0 decides: RCCL when the PS shards live on GPUs, gloo (host buffers) otherwise
            kv.set("ps/pg_backend", "nccl" if device.type == "cuda" else "gloo")
            kv.set("ps/pg_addr", f"127.0.0.1:{_free_port()}")
        self.backend = kv.get("ps/pg_backend").decode()
        if self.backend == "nccl" and device.type != "cuda":
            raise RuntimeError("PS shards are on GPUs (RCCL transport) but this task has no GPU")
        self.comm_device = device if self.backend == "nccl" else torch.device("cpu")
        addr = kv.get("ps/pg_addr").decode()
        kw = {}
        if self.backend == "nccl":
            os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
            kw["device_id"] = device
        if not dist.is_initialized():
            dist.init_process_group(self.backend, init_method=f"tcp://{addr}", rank=self.rank, world_size=self.world,
                                    timeout=datetime.timedelta(seconds=timeout_s), **kw)
        # every rank creates every pair group, in the same order
        self.pairs = {}
        for p in range(self.num_ps):
            for t in range(self.num_trainers):
                g = dist.new_group([p, self.num_ps + t])
                self.pairs[(p, t)] = g

    def trainer_rank(self, t):
        return self.num_ps + t

    def header(self, op=0, n=0):
        return torch.tensor([op, n], dtype=torch.int64, device=self.comm_device)

    def close(self):
        if dist.is_initialized():
            dist.destroy_process_group()


class PSServerLoop:
    """PS side: one thread per trainer serving requests against the shard held by `ps` (ParameterServer)."""

    def __init__(self, ps, group: PSGroup):
        self.ps, self.g = ps, group
        self.lock = threading.Lock()
        self.errors = []

    def _serve(self, t):
        g = self.g
        pg = g.pairs[(self.ps.index, t)]
        src = g.trainer_rank(t)
        dev = g.comm_device
        n_local = self.ps.numel
        hdr = g.header()
        buf = torch.empty(max(1, n_local), dtype=torch.float32, device=dev)
        try:
            while True:
                dist.recv(hdr, src=src, group=pg)
                op, n = (int(v) for v in hdr.tolist())
                if op == OP_DONE:
                    break
                if op in (OP_PUSH, OP_ASSIGN):
                    dist.recv(buf[:n], src=src, group=pg)
                    with self.lock:
                        self.ps.apply_local(buf[:n].to(self.ps.device), assign=(op == OP_ASSIGN))
                        out = self.ps.params_local().to(dev).contiguous()
                    dist.send(out, dst=src, group=pg)
                elif op == OP_PULL:
                    with self.lock:
                        out = self.ps.params_local().to(dev).contiguous()
                    dist.send(out, dst=src, group=pg)
                elif op == OP_SLOTS:
                    with self.lock:
                        slots = [s.to(dev).contiguous() for s in self.ps.slots_local()]
                    for s in slots:
                        dist.send(s, dst=src, group=pg)
        except Exception as e:  # surface in serve()
            self.errors.append(e)

    def run(self):
        ths = [threading.Thread(target=self._serve, args=(t,), daemon=True) for t in range(self.g.num_trainers)]
        for th in ths:
            th.start()
        for th in ths:
            th.join()
        if self.errors:
            raise self.errors[0]


class PSClientGroup:
    """Trainer side: shard-parallel requests to every PS over the pair groups."""

    def __init__(self, group: PSGroup, trainer_index, sizes):
        self.g, self.t, self.sizes = group, trainer_index, sizes
        self.hdrs = [group.header() for _ in sizes]

    def _req(self, op, payloads, recv_bufs):
        works = []
        for p, n in enumerate(self.sizes):
            if n == 0 and op != OP_DONE:
                continue
            pg = self.g.pairs[(p, self.t)]
            self.hdrs[p].copy_(torch.tensor([op, n], dtype=torch.int64))
            works.append(dist.isend(self.hdrs[p], dst=p, group=pg))
            if payloads is not None:
                works.append(dist.isend(payloads[p], dst=p, group=pg))
            if recv_bufs is not None:
                for b in recv_bufs[p]:
                    works.append(dist.irecv(b, src=p, group=pg))
        for w in works:
            w.wait()

    def push(self, grads, params_out):
        """grads[p]: this trainer's gradient slice for shard p; params_out[p] receives the updated values."""
        self._req(OP_PUSH, grads, [[b] for b in params_out])

    def assign(self, values, params_out):
        self._req(OP_ASSIGN, values, [[b] for b in params_out])

    def pull(self, params_out):
        self._req(OP_PULL, None, [[b] for b in params_out])

    def pull_slots(self, slot_bufs):
        self._req(OP_SLOTS, None, slot_bufs)

    def done(self):
        self._req(OP_DONE, None, None)
