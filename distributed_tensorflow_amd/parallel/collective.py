"""Collectives for data parallelism: RCCL over xGMI (GPU) / gloo (CPU).

TF's CollectiveAllReduce (MultiWorkerMirroredStrategy) is realised as
one-process-per-GPU ``torch.distributed`` with the ``nccl`` backend, which is
RCCL on ROCm; on an 8x MI355X node RCCL drives the 7 point-to-point xGMI links
of each GPU.

``GradientBucketer`` overlaps the gradient all-reduce with the backward pass:
the flat gradient arena (see variables.ParamArena) is cut into contiguous
buckets in REVERSE variable order (the order backward produces gradients), a
post-accumulate hook per variable counts arrivals, and a bucket's all-reduce
is issued the moment its last gradient lands — strictly in bucket order, so
every rank issues identical collectives in identical order. Buckets are plain
slices of the arena: no pack/unpack copies. The default
bucket cap is 32 MiB: large enough that a ring over point-to-point xGMI links
runs near link bandwidth, small enough that the first bucket launches while
most of the backward pass is still ahead (SURVEY §5 bandwidth math).
"""
from __future__ import annotations

import datetime
import os

import torch
import torch.distributed as dist

_DEFAULT_BUCKET_MB = float(os.environ.get("DTF_BUCKET_MB", "32"))
# wire dtype of the gradient all-reduce: "f32" (default) or "bf16" (half the bytes on the xGMI links; each
# bucket is cast to bf16 before and back to f32 after the collective, the optimizer still accumulates in f32)
_DEFAULT_WIRE = os.environ.get("DTF_ALLREDUCE_DTYPE", "f32")


def backend_for(device_type: str) -> str:
    """RCCL ("nccl" on ROCm) for GPU replicas, gloo for CPU. ``DTF_COLLECTIVE_BACKEND=gloo`` forces gloo for
    GPU tensors too: it lets several ranks share ONE GPU (RCCL refuses duplicate devices), which is how the
    multi-process GPU data path is rehearsed on a 1-GPU box (tests/test_dp_gpu.py)."""
    forced = os.environ.get("DTF_COLLECTIVE_BACKEND")
    if forced:
        return forced
    return "nccl" if device_type == "cuda" else "gloo"


def init_process_group(rank, world_size, master_addr="127.0.0.1", master_port=29500, device_type=None,
                       timeout_s=600):
    """Initialise (once) the default process group: RCCL for GPUs, gloo for CPUs."""
    if dist.is_initialized():
        return dist.group.WORLD
    if device_type is None:
        device_type = "cuda" if torch.cuda.is_available() else "cpu"
    be = backend_for(device_type)
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    kw = {}
    if be == "nccl":
        kw["device_id"] = torch.device("cuda", torch.cuda.current_device())
    dist.init_process_group(be, init_method=f"tcp://{master_addr}:{master_port}", rank=rank,
                            world_size=world_size, timeout=datetime.timedelta(seconds=timeout_s), **kw)
    return dist.group.WORLD


def world():
    return (dist.get_rank(), dist.get_world_size()) if dist.is_initialized() else (0, 1)


class GradientBucketer:
    """Bucketed, backward-overlapped SUM all-reduce of a ParamArena's gradient buffer."""

    def __init__(self, arena, group=None, bucket_mb=None, average=False, wire_dtype=None, collective=True,
                 implementation=None):
        self.arena = arena
        self.group = group
        # collective=False: no all-reduce (one replica) — the bucketer only drives the per-bucket optimizer update
        self.collective = collective
        self._opt = None        # optimizer whose update runs bucket by bucket during backward (begin_step)
        self.updated = False
        self.average = average
        self.wire = (wire_dtype or _DEFAULT_WIRE).lower()
        if self.wire not in ("f32", "bf16"):
            raise ValueError(f"all-reduce wire dtype {self.wire!r} (f32 or bf16)")
        self._wirebuf = None
        # exposed-communication timing (bench): events around the wait for the last buckets, per step
        self.timing = False
        self._timed = []
        self.bucket_mb = float(bucket_mb if bucket_mb is not None else _DEFAULT_BUCKET_MB)
        cap = int(self.bucket_mb * (1 << 20) / 4)
        nv = len(arena.variables)
        self.buckets = []          # [start, end) element ranges of arena.grad
        self.var_bucket = [0] * nv
        cur_vars, cur_size = [], 0
        for i in reversed(range(nv)):
            cur_vars.append(i)
            cur_size += arena.variables[i].numel()
            if cur_size >= cap:
                self._close(cur_vars)
                cur_vars, cur_size = [], 0
        if cur_vars:
            self._close(cur_vars)
        self.pending = [0] * len(self.buckets)
        self._counts = [0] * len(self.buckets)
        for i in range(nv):
            self._counts[self.var_bucket[i]] += 1
        self._handles = []
        self._works = [None] * len(self.buckets)
        self._next = 0
        self._ready = [False] * len(self.buckets)
        self.enabled = True
        # small buckets (<= p2p.MAX_BYTES) on one node: the one-shot P2P all-reduce over IPC-mapped peer arenas
        # instead of RCCL (collective setup: every rank constructs its bucketer at the same point)
        self.p2p = None
        self.rccl = None  # the framework's own RCCL communicator (rccl.RcclCommunicator), else torch's process group
        self.paths = {"rccl": 0, "p2p": 0, "rccl_native": 0}
        if collective and arena.grad.is_cuda and dist.get_backend(group) == "nccl":
            from . import rccl
            if rccl.wanted(implementation):
                try:
                    self.rccl = rccl.RcclCommunicator(group, device=arena.grad.device)
                except (RuntimeError, OSError, ValueError) as e:
                    print(f"[dtf] native RCCL communicator unavailable ({e}); torch.distributed for the buckets",
                          flush=True)
        if collective and arena.grad.is_cuda and self.rccl is None:
            # process-group collectives order through Work.wait() on RCCL's own stream: hipGraph capture keeps the
            # single multi-branch graph for this configuration
            from ..ops._util import block_split_capture
            block_split_capture(self)
        if collective and arena.grad.is_cuda and self.wire == "f32" and type(self) is GradientBucketer:
            from . import p2p
            spans = [(lo, hi) for lo, hi in self.buckets if (hi - lo) * 4 <= p2p.MAX_BYTES]
            if p2p.available(arena.grad, group) and spans:
                try:
                    self.p2p = p2p.P2PAllReducer(arena.grad, group, spans=spans)
                except (RuntimeError, OSError, ValueError) as e:  # e.g. ranks on several nodes: RCCL only
                    print(f"[dtf] P2P all-reduce unavailable ({e}); RCCL for every bucket", flush=True)
        self.reset()

    def _close(self, var_idx):
        b = len(self.buckets)
        lo = min(self.arena.offsets[i] for i in var_idx)
        last = max(var_idx)
        hi = self.arena.offsets[last + 1] if last + 1 < len(self.arena.offsets) else self.arena.numel
        self.buckets.append((lo, hi))
        for i in var_idx:
            self.var_bucket[i] = b

    def reset(self):
        self.pending = list(self._counts)
        self._ready = [False] * len(self.buckets)
        self._works = [None] * len(self.buckets)
        self._next = 0

    def install(self):
        for i, v in enumerate(self.arena.variables):
            h = v.register_post_accumulate_grad_hook(lambda p, i=i: self._on_grad(i))
            self._handles.append(h)
        return self

    def remove(self):
        for h in self._handles:
            h.remove()
        self._handles = []

    def close(self):
        """Tear the bucketer down: hooks off and the native communicator released (a collective: every rank of the
        group closes its bucketer at the same point, after the last step)."""
        self.remove()
        if self.rccl is not None:
            self.rccl.destroy()
            self.rccl = None

    def _on_grad(self, i):
        if not self.enabled:
            return
        b = self.var_bucket[i]
        self.pending[b] -= 1
        if self.pending[b] == 0:
            self._ready[b] = True
            self._launch_ready()

    def _launch_ready(self):
        while self._next < len(self.buckets) and self._ready[self._next]:
            self._launch(self._next)
            self._next += 1

    def _use_p2p(self, lo, hi):
        if self.p2p is None:
            return False
        from . import p2p
        return (hi - lo) * 4 <= p2p.MAX_BYTES and not torch.cuda.is_current_stream_capturing()

    def begin_step(self, optimizer, grad_scale):
        """Overlap the optimizer with backward: every bucket is updated (masters, slots, bf16 copies, gradient
        zeroing: one fused launch over the bucket's arena range) as soon as its gradients are final — right after
        its all-reduce, or when its last gradient lands with one replica — on a stream of its own, while backward
        continues. The update of the last buckets is all that remains after backward (SURVEY §2.6 overlap)."""
        optimizer.set_grad_scale(grad_scale)
        optimizer.begin_step(self.arena)
        self._opt = optimizer

    def _launch(self, b):
        lo, hi = self.buckets[b]
        t = self.arena.grad[lo:hi]
        import contextlib
        work = None
        if self.collective and self._use_p2p(lo, hi):
            # one kernel on the communication stream (it waits for the main and weight-gradient streams as they are
            # now): stream-ordered, no Work to wait on, and a spin on a late peer stalls no weight-gradient GEMM
            from ..ops._util import comm_stream_ctx
            with comm_stream_ctx(t.device):
                self.p2p.all_reduce_(lo, hi)
            self.paths["p2p"] += 1
        elif self.collective and self.rccl is not None:
            # the native communicator: stream-ordered on the communication stream (it waits for the main and
            # weight-gradient streams as they are now), so neither compute stream waits for the collective
            from ..ops._util import comm_stream_ctx
            with comm_stream_ctx(t.device):
                if self.wire == "bf16":
                    if self._wirebuf is None:
                        self._wirebuf = torch.empty(self.arena.grad.numel(), dtype=torch.bfloat16, device=t.device)
                    _cast(t, self._wirebuf[lo:hi])
                    self.rccl.all_reduce_(self._wirebuf[lo:hi])
                    _cast(self._wirebuf[lo:hi], t)
                else:
                    self.rccl.all_reduce_(t)
            self.paths["rccl_native"] += 1
        elif self.collective:
            ctx = contextlib.nullcontext()
            if t.is_cuda:  # the bucket's weight gradients may still be in flight on the side stream
                from ..ops._util import collective_ctx
                ctx = collective_ctx(t.device)
            with ctx:
                self.paths["rccl"] += 1
                if self.wire == "bf16":
                    if self._wirebuf is None:
                        self._wirebuf = torch.empty(self.arena.grad.numel(), dtype=torch.bfloat16, device=t.device)
                    w = self._wirebuf[lo:hi]
                    _cast(t, w)
                    t = w
                work = dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group, async_op=True)
        if self._opt is None:
            self._works[b] = work
            return
        uctx = contextlib.nullcontext()
        if t.is_cuda:
            from ..ops._util import update_stream_ctx
            uctx = update_stream_ctx(t.device)
        with uctx:
            if work is not None:
                work.wait()  # GPU: the update stream waits for the collective (the host does not)
                if self.wire == "bf16":
                    _cast(self._wirebuf[lo:hi], self.arena.grad[lo:hi])
            if self.average and self.collective:
                self.arena.grad[lo:hi].div_(dist.get_world_size(self.group))
            self._opt.apply_range(self.arena, lo, hi)

    def finalize(self):
        """Issue buckets whose variables got no gradient (in order), then wait for all of them."""
        # buckets the post-accumulate hooks launched DURING backward (the overlap actually happened)
        self.launched_in_backward = self._next
        if self.arena.grad.is_cuda:
            from ..ops._util import join_side_streams
            join_side_streams()
        while self._next < len(self.buckets):
            self._launch(self._next)
            self._next += 1
        ev0 = None
        if self.timing and self.arena.grad.is_cuda and not torch.cuda.is_current_stream_capturing():
            ev0 = torch.cuda.Event(enable_timing=True)
            ev0.record()  # backward compute is done here; what follows on this stream is waiting on RCCL
        if self._opt is not None:
            # every bucket was updated on the update stream: the step's tail is its last updates
            if self.arena.grad.is_cuda:
                from ..ops._util import join_update_stream
                join_update_stream(self.arena.grad.device)
            self._opt = None
            self.updated = True
        else:
            for w in self._works:
                if w is not None:
                    w.wait()  # GPU: the main stream waits for the collective's RCCL stream
            if self.arena.grad.is_cuda:
                from ..ops._util import join_comm_stream
                join_comm_stream(self.arena.grad.device)  # P2P / native RCCL buckets ran on the comm stream
                if self.p2p is not None:
                    self.p2p.poll()
            if self.wire == "bf16" and self.collective and self.rccl is None:
                for lo, hi in self.buckets:
                    _cast(self._wirebuf[lo:hi], self.arena.grad[lo:hi])
            if self.average and self.collective:
                self.arena.grad.div_(dist.get_world_size(self.group))
        if ev0 is not None:
            ev1 = torch.cuda.Event(enable_timing=True)
            ev1.record()
            self._timed.append((ev0, ev1))
        self.reset()

    def exposed_ms(self, clear=True):
        """Mean device time per timed step between the end of the backward compute and the completion of the
        last gradient bucket (communication the backward overlap did not hide); None if nothing was timed."""
        if not self._timed:
            return None
        torch.cuda.synchronize()
        v = sum(a.elapsed_time(b) for a, b in self._timed) / len(self._timed)
        if clear:
            self._timed = []
        return v


class ShardedGradientBucketer(GradientBucketer):
    """ZeRO-1 data parallelism: the optimizer update is sharded across the replicas.

    Same buckets, hooks and issue order as GradientBucketer, but each bucket is REDUCE-SCATTERED instead of
    all-reduced: bucket [lo, hi) of length L is cut into ``world`` chunks of s = ceil(L / world) elements and
    rank r receives the summed chunk r in a compact shard-gradient buffer. After backward every rank runs the
    fused optimizer kernel over its own chunks only (1/world of the update's HBM traffic — for Adam that is
    ~26 B/param of the step), then the updated f32 masters are ALL-GATHERED back bucket by bucket and the bf16
    compute copies refreshed from them. The bytes on the xGMI links equal the all-reduce's (a ring all-reduce
    IS a reduce-scatter + all-gather); the saving is the replicated optimizer work.

    Optimizer slots keep their full-arena layout but only the owned chunks are current on each rank;
    ``gather_slots()`` (a collective: every rank must call it) all-gathers them before a checkpoint is written.
    LAMB's per-variable trust ratio does not decompose over chunks and is rejected.
    SURVEY §2.6 "Reduce-scatter / all-gather (ZeRO-1, optional)".
    """

    def __init__(self, arena, group=None, bucket_mb=None, wire_dtype=None, implementation=None):
        super().__init__(arena, group=group, bucket_mb=bucket_mb, wire_dtype=wire_dtype, implementation=implementation)
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.shards = []   # per bucket: (chunk s, own_lo, own_hi, compact offset)
        off = 0
        for lo, hi in self.buckets:
            s = -(-(hi - lo) // self.world)
            s = -(-s // 16) * 16  # 64-B aligned chunks: the fused update runs 16-B vector loads on every segment
            own_lo = min(hi, lo + self.rank * s)
            own_hi = min(hi, own_lo + s)
            self.shards.append((s, own_lo, own_hi, off))
            off += s
        dev = arena.grad.device
        self.sgrad = torch.zeros(off, dtype=torch.float32, device=dev)   # this rank's summed gradient chunks
        wire_t = torch.bfloat16 if self.wire == "bf16" else torch.float32
        # padded send images for buckets whose length is not a multiple of world (or bf16 wire), zero tails
        self._send = {}
        self._recv = {}
        for b, (lo, hi) in enumerate(self.buckets):
            s = self.shards[b][0]
            if self.wire == "bf16" or (hi - lo) != s * self.world:
                self._send[b] = torch.zeros(s * self.world, dtype=wire_t, device=dev)
            if self.wire == "bf16":
                self._recv[b] = torch.zeros(s, dtype=wire_t, device=dev)
        self._gather = {}  # padded all-gather images (f32), allocated on first use

    def _launch(self, b):
        lo, hi = self.buckets[b]
        s, _, _, c = self.shards[b]
        import contextlib
        ctx = contextlib.nullcontext()
        g = self.arena.grad[lo:hi]
        if g.is_cuda:
            from ..ops._util import collective_ctx, comm_stream_ctx
            # native communicator: stream-ordered on the communication stream (hipGraph-capturable, no Work)
            ctx = comm_stream_ctx(g.device) if self.rccl is not None else collective_ctx(g.device)
        with ctx:
            inp = g
            if b in self._send:
                inp = self._send[b]
                if self.wire == "bf16":
                    _cast(g, inp[:hi - lo])
                else:
                    inp[:hi - lo].copy_(g)
            out = self._recv.get(b, self.sgrad[c:c + s])
            if self.rccl is not None:
                self.rccl.reduce_scatter(inp, out)
                self.paths["rccl_native"] += 1
            else:
                self._works[b] = dist.reduce_scatter_tensor(out, inp, op=dist.ReduceOp.SUM, group=self.group,
                                                            async_op=True)
                self.paths["rccl"] += 1

    def finalize(self):
        if self.arena.grad.is_cuda:
            from ..ops._util import join_side_streams
            join_side_streams()
        while self._next < len(self.buckets):
            self._launch(self._next)
            self._next += 1
        ev0 = None
        if self.timing and self.arena.grad.is_cuda and not torch.cuda.is_current_stream_capturing():
            ev0 = torch.cuda.Event(enable_timing=True)
            ev0.record()
        for w in self._works:
            if w is not None:
                w.wait()
        if self.rccl is not None and self.arena.grad.is_cuda:
            from ..ops._util import join_comm_stream
            join_comm_stream(self.arena.grad.device)
        for b, r in self._recv.items():
            s, _, _, c = self.shards[b]
            _cast(r, self.sgrad[c:c + s])
        if ev0 is not None:
            ev1 = torch.cuda.Event(enable_timing=True)
            ev1.record()
            self._timed.append((ev0, ev1))
        # the replicated gradient arena has been consumed (the update reads the compact chunks): clear it for
        # the next backward's accumulation
        self.arena.grad.zero_()
        self.reset()

    def segments(self):
        """(own_lo, own_hi, compact gradient view) of every bucket this rank updates."""
        out = []
        for s, lo, hi, c in self.shards:
            if hi > lo:
                out.append((lo, hi, self.sgrad[c:c + hi - lo]))
        return out

    def _all_gather_(self, buf):
        """In-place all-gather of this rank's chunks of ``buf`` (an arena-shaped f32 buffer), bucket by bucket."""
        if self.rccl is not None:
            return self._all_gather_native(buf)
        works = []
        for b, (lo, hi) in enumerate(self.buckets):
            s, own_lo, own_hi, _ = self.shards[b]
            if (hi - lo) == s * self.world:
                # NCCL/RCCL in-place form: the input is the rank's own slice of the output
                works.append((None, dist.all_gather_into_tensor(buf[lo:hi], buf[own_lo:own_lo + s],
                                                                group=self.group, async_op=True)))
            else:
                img = self._gather.get(b)
                if img is None:
                    img = self._gather[b] = torch.zeros(s * self.world, dtype=buf.dtype, device=buf.device)
                mine = torch.zeros(s, dtype=buf.dtype, device=buf.device)
                mine[:own_hi - own_lo].copy_(buf[own_lo:own_hi])
                works.append((b, dist.all_gather_into_tensor(img, mine, group=self.group, async_op=True)))
        for b, w in works:
            w.wait()
            if b is not None:
                lo, hi = self.buckets[b]
                buf[lo:hi].copy_(self._gather[b][:hi - lo])

    def _all_gather_native(self, buf):
        """_all_gather_ on the framework's communicator, stream-ordered on the current stream."""
        for b, (lo, hi) in enumerate(self.buckets):
            s, own_lo, own_hi, _ = self.shards[b]
            if (hi - lo) == s * self.world:
                self.rccl.all_gather(buf[own_lo:own_lo + s], buf[lo:hi])  # in place: the input is our slice
            else:
                img = self._gather.get(b)
                if img is None:
                    img = self._gather[b] = torch.zeros(s * self.world, dtype=buf.dtype, device=buf.device)
                mine = img[self.rank * s:(self.rank + 1) * s]
                mine.zero_()
                mine[:own_hi - own_lo].copy_(buf[own_lo:own_hi])
                self.rccl.all_gather(mine, img)
                buf[lo:hi].copy_(img[:hi - lo])

    def gather_params(self):
        """All-gather the updated f32 masters and refresh the bf16 compute copies."""
        self._all_gather_(self.arena.flat)
        if self.arena.bf16 is not None:
            _cast(self.arena.flat, self.arena.bf16)

    def gather_slots(self, optimizer):
        """Make every optimizer slot current on every rank (collective; call on all ranks before a save)."""
        for nm, _ in optimizer.slot_specs():
            self._all_gather_(self.arena.slots[nm])


def _cast(src, dst):
    """f32 <-> bf16 conversion of one bucket (HIP cast kernels on GPU)."""
    if src.is_cuda:
        from ..ops._util import call, stream
        name = "dtf_cast_f32_bf16" if src.dtype == torch.float32 else "dtf_cast_bf16_f32"
        call(name, src.data_ptr(), dst.data_ptr(), src.numel(), stream())
    else:
        dst.copy_(src)


class ShmAllReduce:
    """Host shared-memory all-reduce (csrc/runtime/shm_allreduce.cc) for CPU gradient arenas of
    processes on one node: one reduce-scatter/all-gather through /dev/shm per step instead of gloo's
    loopback TCP. Used by MultiWorkerMirroredStrategy on CPU when DTF_CPU_ALLREDUCE=shm (default)."""

    def __init__(self, arena, rank, world, name):
        from .. import _native
        from .._runtime_sigs import err
        self.lib = _native.runtime()
        self.arena = arena
        nbytes = min(arena.grad.numel() * 4, 64 << 20)
        self.h = self.lib.dtfrt_shm_open(name.encode(), rank, world, nbytes)
        if not self.h:
            raise OSError(err(self.lib))
        self.rank = rank

    def install(self):
        return self

    def finalize(self):
        g = self.arena.grad
        if self.lib.dtfrt_shm_allreduce_f32(self.h, g.data_ptr(), g.numel()) != 0:
            raise RuntimeError("shared-memory all-reduce timed out")

    def close(self):
        if self.h:
            self.lib.dtfrt_shm_close(self.h, int(self.rank == 0))
            self.h = None


def broadcast_tensors(tensors, src=0, group=None):
    for t in tensors:
        dist.broadcast(t, src=src, group=group)


def all_reduce_(t, op="sum", group=None):
    ops = {"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX, "min": dist.ReduceOp.MIN}
    if op == "mean":
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
        t.div_(dist.get_world_size(group))
    else:
        dist.all_reduce(t, op=ops[op], group=group)
    return t
