"""tf.distribute-style strategies on MI355X.

* ``OneDeviceStrategy`` / default strategy — single device.
* ``MirroredStrategy`` — synchronous data parallelism. Under a one-process-per-GPU
  launch (torchrun / bench.py, the idiomatic MI355X layout) it is the same
  collective all-reduce as MultiWorkerMirroredStrategy restricted to one node.
  Given several local devices in ONE process it runs in-process replicas
  (``CPU:0,CPU:1`` plumbing config of BASELINE.json): replicas share the
  variables when they share a device, otherwise gradients are reduced to the
  first device (ReductionToOneDevice) and weights broadcast back.
* ``MultiWorkerMirroredStrategy`` — CollectiveAllReduce across processes,
  topology from TF_CONFIG (chief/worker tasks) or torchrun's env, RCCL over
  xGMI for GPUs and gloo for CPUs, with the bucketed backward-overlapped
  all-reduce of ``collective.GradientBucketer``.
* ``ParameterServerStrategy`` lives in ``parameter_server.py``.
"""
from __future__ import annotations

import contextlib
import enum
import os
import threading

import torch
import torch.distributed as dist

from .. import context
from . import collective
from .cluster_resolver import TFConfigClusterResolver, TorchrunClusterResolver

_tls = threading.local()

# The optimizer update can run bucket by bucket during backward (GradientBucketer.begin_step) on a stream of its
# own. DTF_OVERLAP_UPDATE: unset = the model's choice (Model.overlap_update), "0" off, "1" on, "force" on also for
# CPU arenas (tests). Measured on one MI355X: GPT-2-medium fp8 +2% (34.84 vs 35.58 ms; its data-gradient chain
# leaves CUs idle), bf16 GPT-2-medium -1%, ResNet-50 -0.8%, BERT-base +-0 (backward already keeps every CU busy:
# the memory-bound update only moves, it does not hide).
_OVERLAP_UPDATE = os.environ.get("DTF_OVERLAP_UPDATE", "")
# A hipGraph-captured step never takes the per-bucket update (round-4 bisection, tools/debug_r4.py capture: bucket
# updates issued from autograd's post-accumulate hooks during the capture replay differently from eager — with the
# update on its own stream the stem's bucket diverges from the first replay, with the update on the capture stream
# (or the weight gradients on the main stream) the first replay's forward already differs — while the same buckets
# updated after backward (finalize) replay bit-identically; the optimizer is one ~120 us launch per ResNet-50 step,
# so the capture keeps the single fused update after backward). The per-stream capture (graphs.py, split) records the
# update stream as a graph of its own with explicit event / flag edges and keeps the per-bucket update.


class ReduceOp(enum.Enum):
    SUM = "sum"
    MEAN = "mean"
    MAX = "max"
    MIN = "min"


def get_strategy():
    s = getattr(_tls, "strategy", None)
    return s if s is not None else _default()


def has_strategy():
    return getattr(_tls, "strategy", None) is not None


_DEFAULT = None


def _default():
    global _DEFAULT
    if _DEFAULT is None:
        _DEFAULT = OneDeviceStrategy(context.default_device())
    return _DEFAULT


class Strategy:
    """Common interface the Keras training loop talks to."""

    def __init__(self):
        self._bucketers = {}

    # ---- properties
    @property
    def num_replicas_in_sync(self):
        return 1

    @property
    def is_chief(self):
        return True

    @property
    def worker_index(self):
        return 0

    @property
    def num_workers(self):
        return 1

    @property
    def device(self):
        return context.default_device()

    @contextlib.contextmanager
    def scope(self):
        prev = getattr(_tls, "strategy", None)
        _tls.strategy = self
        try:
            with context.device(self.device):
                yield self
        finally:
            _tls.strategy = prev

    # ---- training-loop hooks
    def order_variables(self, variables):
        """The order of the trainable variables in the model's parameter arena (identity by default;
        ParameterServerStrategy groups them by PS shard)."""
        return list(variables)

    def setup_model(self, model, arena):
        """Called once after the trainable arena exists (broadcast initial state, install hooks)."""

    def _overlap_bucketer(self, arena, optimizer):
        """The bucketer that runs ``optimizer`` bucket by bucket during backward, or None (CPU arenas, global-norm
        clipping, sharded or in-process-replica updates)."""
        if optimizer is None or _OVERLAP_UPDATE == "0" or not optimizer.supports_ranges():
            return None
        if not arena.grad.is_cuda and _OVERLAP_UPDATE != "force":
            return None
        if arena.grad.is_cuda and torch.cuda.is_current_stream_capturing():
            from ..ops import _util
            if _util._SPLIT is None:
                return None  # a single-graph capture keeps the single update after backward (see above)
        b = self._bucketers.get(id(arena))
        if b is None:  # one replica: a bucketer without collectives, only to time the bucket updates
            b = collective.GradientBucketer(arena, collective=False).install()
            self._bucketers[id(arena)] = b
        return b if type(b) is collective.GradientBucketer else None

    def backward(self, loss, arena, optimizer=None):
        b = self._overlap_bucketer(arena, optimizer)
        if b is not None:
            b.begin_step(optimizer, self.grad_scale())
        loss.backward()
        if b is not None:
            b.finalize()

    def grad_scale(self):
        return 1.0

    def apply_gradients(self, optimizer, arena):
        """Apply the (already reduced) gradient arena: one fused optimizer launch — or, when the update already
        ran bucket by bucket during backward, only close the step."""
        b = self._bucketers.get(id(arena))
        if b is not None and getattr(b, "updated", False):
            b.updated = False
            optimizer.end_step(arena)
            return
        optimizer.set_grad_scale(self.grad_scale())
        optimizer.apply_arena(arena, zero_grad=True)

    def local_batch_slice(self, n):
        """Which rows of a global batch of n rows this process consumes."""
        return slice(0, n)

    def reduce(self, op, value, axis=None):
        v = value
        if axis is not None and isinstance(v, torch.Tensor):
            v = v.sum(axis) if _op(op) == "sum" else v.mean(axis)
        return v

    def run(self, fn, args=(), kwargs=None):
        return fn(*args, **(kwargs or {}))

    def experimental_distribute_dataset(self, dataset):
        return dataset

    def distribute_datasets_from_function(self, fn):
        return fn(InputContext(self.num_workers, self.worker_index, self.num_replicas_in_sync))

    def barrier(self):
        pass


def _op(op):
    return op.value if isinstance(op, ReduceOp) else str(op).lower()


class InputContext:
    def __init__(self, num_input_pipelines, input_pipeline_id, num_replicas_in_sync):
        self.num_input_pipelines = num_input_pipelines
        self.input_pipeline_id = input_pipeline_id
        self.num_replicas_in_sync = num_replicas_in_sync

    def get_per_replica_batch_size(self, global_batch_size):
        if global_batch_size % self.num_replicas_in_sync:
            raise ValueError("global batch size must be divisible by the number of replicas")
        return global_batch_size // self.num_replicas_in_sync


class OneDeviceStrategy(Strategy):
    def __init__(self, device=None):
        super().__init__()
        self._device = context.parse_device(device) if device is not None else context.default_device()

    @property
    def device(self):
        return self._device


class CommunicationImplementation(enum.Enum):
    """tf.distribute.experimental.CommunicationImplementation. On GPUs every choice is RCCL over xGMI: NCCL drives
    the framework's own communicator (parallel/rccl.py, C++ csrc/runtime/rccl_comm.cc, channel count set at
    creation), RING torch.distributed's ProcessGroupNCCL, AUTO the former unless DTF_COMM=torch. CPU replicas use
    gloo / the shared-memory all-reduce whatever is asked."""
    AUTO = "AUTO"
    RING = "RING"
    NCCL = "NCCL"


class CommunicationOptions:
    """tf.distribute.experimental.CommunicationOptions: ``bytes_per_pack`` is the gradient bucket cap (0 = the
    framework default, DTF_BUCKET_MB); ``implementation`` a CommunicationImplementation; ``wire_dtype`` ("f32" /
    "bf16", an extension) the all-reduce payload type."""

    def __init__(self, bytes_per_pack=0, timeout_seconds=None, implementation=CommunicationImplementation.AUTO,
                 wire_dtype=None):
        self.bytes_per_pack = int(bytes_per_pack or 0)
        self.timeout_seconds = timeout_seconds
        if isinstance(implementation, str):
            implementation = CommunicationImplementation(implementation.upper())
        self.implementation = implementation
        self.wire_dtype = wire_dtype


class MultiWorkerMirroredStrategy(Strategy):
    """Synchronous collective all-reduce data parallelism, one process per device."""

    shard_optimizer = False

    def __init__(self, cluster_resolver=None, communication_options=None, bucket_mb=None, shard_optimizer=None):
        super().__init__()
        # ZeRO-1 (collective.ShardedGradientBucketer): reduce-scatter gradients, update 1/N of the arena per
        # replica, all-gather the masters; DTF_ZERO=1 turns it on without code changes
        self.shard_optimizer = bool(int(os.environ.get("DTF_ZERO", "0"))) if shard_optimizer is None \
            else bool(shard_optimizer)
        co = communication_options
        if bucket_mb is None and co is not None and co.bytes_per_pack:
            bucket_mb = co.bytes_per_pack / float(1 << 20)
        self.wire_dtype = getattr(co, "wire_dtype", None)
        impl = getattr(co, "implementation", None)
        self.implementation = None if impl in (None, CommunicationImplementation.AUTO) else impl
        self.bucket_mb = bucket_mb
        if cluster_resolver is None:
            if TorchrunClusterResolver.active():
                cluster_resolver = TorchrunClusterResolver()
            else:
                cluster_resolver = TFConfigClusterResolver()
        self.cluster_resolver = cluster_resolver
        if isinstance(cluster_resolver, TorchrunClusterResolver):
            self._rank, self._world = cluster_resolver.rank, cluster_resolver.world_size
            addr, port = cluster_resolver.master_addr, cluster_resolver.master_port
            self._local_rank = cluster_resolver.local_rank
        else:
            tasks = cluster_resolver.trainer_tasks() if not cluster_resolver.standalone else [("worker", 0)]
            self._world = len(tasks)
            self._rank = max(0, cluster_resolver.trainer_rank()) if not cluster_resolver.standalone else 0
            chief_addr = cluster_resolver.cluster.task_address(*tasks[0]) if not cluster_resolver.standalone \
                else "127.0.0.1:29500"
            addr, port = chief_addr.rsplit(":", 1)
            port = int(port)
            self._local_rank = int(os.environ.get("LOCAL_RANK", self._rank if torch.cuda.device_count() > 1 else 0))
        if torch.cuda.is_available():
            # the launcher's per-task ordinal (cli.launch --gpus) wins over the rank-derived one
            ordinal = context.local_ordinal(self._local_rank) if "DTF_DEVICE_ORDINAL" in os.environ \
                else self._local_rank
            dev = context.bind_device(torch.device("cuda", ordinal % torch.cuda.device_count()))
        else:
            dev = torch.device("cpu")
        self._device = dev
        # DTF_FORCE_COLLECTIVE=1: run the collective path (process group + bucketed all-reduce) even with one
        # replica — how the RCCL code path and its hipGraph capture are exercised on a 1-GPU box
        self._force = os.environ.get("DTF_FORCE_COLLECTIVE", "0") == "1"
        if self._world > 1 or self._force:
            from ..ops._util import reserve_streams
            reserve_streams(dev)  # the side stream's hardware queue before RCCL's
            collective.init_process_group(self._rank, self._world, addr, port, dev.type)

    @property
    def device(self):
        return self._device

    @property
    def num_replicas_in_sync(self):
        return self._world

    @property
    def num_workers(self):
        return self._world

    @property
    def worker_index(self):
        return self._rank

    @property
    def is_chief(self):
        return self._rank == 0

    def setup_model(self, model, arena):
        if self._world <= 1 and not getattr(self, "_force", False):
            return
        # identical initial state everywhere: one broadcast of the whole master arena + non-trainables
        collective.broadcast_tensors([arena.flat] + [v.data for v in model.non_trainable_weights], src=0)
        arena.refresh_bf16()
        from ..ops._util import bump_weights_epoch
        bump_weights_epoch()
        if self.shard_optimizer:
            b = collective.ShardedGradientBucketer(arena, bucket_mb=self.bucket_mb,
                                                   wire_dtype=getattr(self, "wire_dtype", None),
                                                   implementation=getattr(self, "implementation", None)).install()
        elif arena.grad.device.type == "cpu" and os.environ.get("DTF_CPU_ALLREDUCE", "shm") == "shm":
            # one node, CPU arenas: shared-memory reduce-scatter/all-gather instead of gloo TCP
            name = f"ar{os.environ.get('MASTER_PORT', '0')}_{len(self._bucketers)}"
            if dist.get_rank() == 0:
                import secrets
                name += "_" + secrets.token_hex(4)
            obj = [name]
            dist.broadcast_object_list(obj, src=0)
            b = collective.ShmAllReduce(arena, self._rank, self._world, obj[0])
        else:
            b = collective.GradientBucketer(arena, bucket_mb=self.bucket_mb,
                                            wire_dtype=getattr(self, "wire_dtype", None),
                                            implementation=getattr(self, "implementation", None)).install()
        self._bucketers[id(arena)] = b

    def backward(self, loss, arena, optimizer=None):
        if getattr(self, "_inproc", False):
            return Strategy.backward(self, loss, arena)
        ob = self._overlap_bucketer(arena, optimizer)
        if ob is not None:
            ob.begin_step(optimizer, self.grad_scale())
        loss.backward()
        b = self._bucketers.get(id(arena))
        if b is not None:
            b.finalize()

    def grad_scale(self):
        return 1.0 / self._world

    def apply_gradients(self, optimizer, arena):
        b = self._bucketers.get(id(arena))
        if not isinstance(b, collective.ShardedGradientBucketer):
            return Strategy.apply_gradients(self, optimizer, arena)
        optimizer.set_grad_scale(self.grad_scale())
        red = (lambda t: b.rccl.all_reduce_(t)) if getattr(b, "rccl", None) is not None else (lambda t: dist.all_reduce(t))
        optimizer.apply_segments(arena, b.segments(), reduce_sumsq=red)
        b.gather_params()

    def sync_optimizer_state(self, optimizer):
        """Collective (every replica calls it): make sharded optimizer slots whole on every replica before a
        checkpoint is written. A no-op unless the optimizer state is sharded (ZeRO-1)."""
        for b in self._bucketers.values():
            if isinstance(b, collective.ShardedGradientBucketer):
                b.gather_slots(optimizer)

    def agree(self, flag, every=16):
        """Rank 0's decision (e.g. a time-based checkpoint trigger) on every replica. The decision is exchanged
        only on every `every`-th call (all replicas count calls identically, so they consult together); on the
        other calls it is False without a collective — no per-batch broadcast + host sync."""
        if self._world <= 1 or not self.shard_optimizer:
            return flag
        self._agree_calls = getattr(self, "_agree_calls", 0) + 1
        if self._agree_calls % max(1, int(every)):
            return False
        t = torch.tensor([1 if flag else 0], dtype=torch.int32, device=self._device)
        dist.broadcast(t, src=0)
        return bool(t.item())

    def local_batch_slice(self, n):
        per = n // self._world
        return slice(self._rank * per, (self._rank + 1) * per)

    def reduce(self, op, value, axis=None):
        v = super().reduce(op, value, axis)
        if self._world <= 1:
            return v
        t = v if isinstance(v, torch.Tensor) else torch.tensor(float(v), device=self._device)
        t = t.detach().clone().to(self._device).float()
        collective.all_reduce_(t, _op(op))
        return t

    def experimental_distribute_dataset(self, dataset):
        return dataset.shard(self._world, self._rank) if self._world > 1 else dataset

    def barrier(self):
        if self._world > 1:
            dist.barrier()


_MIRRORED_CHILD = "DTF_MIRRORED_CHILD"


def _spawn_replicas(devices):
    """The parent side of MirroredStrategy(devices=[GPU...]): run this same program once per device, each copy a
    replica of a multi-process MirroredStrategy (RANK / WORLD_SIZE / LOCAL_RANK / MASTER_* for the process group,
    DTF_DEVICE_ORDINAL for its GPU), wait for them and exit with the worst status. The parent touches no GPU: the
    children are started as plain subprocesses (no exec of the running program).

    Refused (ValueError / RuntimeError) when the program cannot be re-run as-is: ``python -c``, a host test runner
    (pytest would re-run the whole session once per device), or a parent that already initialised HIP. The parent
    polls all children: the first one to fail terminates its siblings (which would otherwise sit in rendezvous or
    RCCL init until their timeout), and SIGINT / SIGTERM sent to the parent are forwarded to every child."""
    import signal
    import socket
    import subprocess
    import sys
    import time
    argv = list(getattr(sys, "orig_argv", []))[1:] or list(sys.argv)
    if not argv or argv[0] == "-c":
        raise ValueError("MirroredStrategy over several GPUs re-runs the program once per GPU: it needs a script or "
                         "module (python script.py / python -m module), not python -c")
    if "pytest" in sys.modules:
        raise ValueError("MirroredStrategy over several GPUs re-runs the program once per GPU; under a test runner "
                         "that would re-run the whole session: start the replicas with cli.launch / torchrun instead")
    if torch.cuda.is_initialized():
        raise RuntimeError("MirroredStrategy over several GPUs must be constructed before the program touches a GPU: "
                           "this process initialised HIP already, and it starts one child process per device")
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []

    def _forward(signum, _frame):
        for p in procs:
            if p.poll() is None:
                p.send_signal(signum)

    prev = {sig: signal.signal(sig, _forward) for sig in (signal.SIGINT, signal.SIGTERM)}
    try:
        for r, d in enumerate(devices):
            env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(len(devices)), LOCAL_RANK=str(r),
                       MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), DTF_DEVICE_ORDINAL=str(d.index or 0))
            env[_MIRRORED_CHILD] = "1"
            procs.append(subprocess.Popen([sys.executable] + argv, env=env))
        rc = 0
        live = list(procs)
        while live:
            for p in list(live):
                code = p.poll()
                if code is None:
                    continue
                live.remove(p)
                if code != 0:
                    rc = max(rc, abs(code))
                    for q in live:  # a dead replica leaves its peers blocked in collectives: stop them
                        q.terminate()
            time.sleep(0.05)
        for p in procs:
            p.wait()
    finally:
        for sig, h in prev.items():
            signal.signal(sig, h)
    raise SystemExit(rc)


class MirroredStrategy(MultiWorkerMirroredStrategy):
    """Single-node synchronous data parallelism (TF's ``MirroredStrategy(devices)``).

    devices=[GPU, GPU, ...]: one replica per listed GPU. On MI355X every GPU gets its own process (its own HIP
    runtime queues, RCCL rank and Python interpreter), so the constructor, called in the parent, re-runs the program
    once per device and exits with their status (``_spawn_replicas``); in each child the same constructor call
    finds its replica through the environment and returns a multi-process strategy bound to its device. Construct
    the strategy before the program touches a GPU (the parent must not initialise HIP). A device may be listed
    twice (two replicas sharing one GPU: the 1-GPU rehearsal of the path, with DTF_COLLECTIVE_BACKEND=gloo).
    devices=None under a multi-process launch (cli.launch --gpus N, torchrun): one replica per process.
    devices=[host devices] in one process: in-process replicas (the reference's CPU:0 / CPU:1 plumbing config)."""

    def __init__(self, devices=None, cross_device_ops=None, bucket_mb=None, communication_options=None,
                 shard_optimizer=None):
        self._devices = [context.parse_device(d) for d in devices] if devices else None
        self.wire_dtype = getattr(communication_options, "wire_dtype", None)
        ngpu = sum(1 for d in (self._devices or []) if d.type == "cuda")
        if ngpu > 1 and not TorchrunClusterResolver.active():
            if ngpu != len(self._devices):
                raise ValueError("MirroredStrategy: mixing GPU and host devices is not supported")
            _spawn_replicas(self._devices)  # (does not return in the parent)
        if ngpu > 1 and os.environ.get(_MIRRORED_CHILD) == "1":
            # a child of _spawn_replicas: the listed device of this rank (DTF_DEVICE_ORDINAL) via the launcher path
            self._inproc = False
            self._devices = None
            super().__init__(TorchrunClusterResolver(), communication_options, bucket_mb=bucket_mb,
                             shard_optimizer=shard_optimizer)
            return
        if self._devices and len(self._devices) > 1 and not TorchrunClusterResolver.active():
            Strategy.__init__(self)
            self.bucket_mb = bucket_mb
            self._rank, self._world, self._local_rank = 0, 1, 0
            self._device = self._devices[0]
            self.cluster_resolver = None
            self._inproc = True
            return
        self._inproc = False
        if self._devices and len(self._devices) == 1:
            Strategy.__init__(self)
            self.bucket_mb = bucket_mb
            self._rank, self._world, self._local_rank = 0, 1, 0
            self._device = self._devices[0]
            self.cluster_resolver = None
            return
        if TorchrunClusterResolver.active():
            super().__init__(TorchrunClusterResolver(), communication_options, bucket_mb=bucket_mb,
                             shard_optimizer=shard_optimizer)
        else:
            super().__init__(TFConfigClusterResolver(tf_config={}), communication_options, bucket_mb=bucket_mb,
                             shard_optimizer=shard_optimizer)

    @property
    def extended_devices(self):
        return self._devices or [self._device]

    @property
    def num_replicas_in_sync(self):
        if self._inproc:
            return len(self._devices)
        return self._world

    # ---- in-process replica execution (used by Model.train_step when _inproc)
    def inproc_replicas(self):
        return self._devices if self._inproc else None

    def grad_scale(self):
        if self._inproc:
            return 1.0 / len(self._devices)
        return super().grad_scale()
