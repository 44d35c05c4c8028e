"""The framework's own RCCL communicator (csrc/runtime/rccl_comm.cc): collectives driven from C++ on streams the
framework chooses, with the channel (CTA) count set at creation.

torch.distributed's ProcessGroupNCCL stays the rendezvous and the fallback; ``RcclCommunicator`` is what the gradient
bucketer drives when ``CommunicationOptions(implementation=CommunicationImplementation.NCCL)`` (or ``DTF_COMM=native``)
asks for it:

* rank 0 draws the 128-byte unique id and publishes it through the process group's store (the C++ TCP store of the
  rendezvous); every rank creates its communicator on its bound GPU with ``ncclCommInitRankConfig``;
* ``min_channels`` (default 8): one ring channel per xGMI link direction — an MI355X has 7 point-to-point links, so
  fewer channels leave links idle on an 8-GPU node; ``max_channels`` (default 16) caps the CUs a collective takes from
  the backward pass it overlaps (one CTA per channel);
* collectives are stream-ordered on the caller's current stream (no Work objects, no host waits), so they run inside
  a hipGraph capture like any kernel;
* a self-check all-reduce at creation (sum of rank + 1 over the group) catches a misconfigured communicator before
  any gradient goes through it.

Reference parity: TF's CollectiveAllReduce on NCCL (/root/reference/trainer/task.py:150-175 builds the strategies that
use it); SURVEY §1.2 "RCCL over xGMI", VERDICT r4 "an RCCL communicator owned by the framework".
"""
from __future__ import annotations

import atexit
import collections
import ctypes
import os
import weakref

import torch

from .. import _native

_DT = {torch.float32: 7, torch.bfloat16: 9, torch.float16: 6, torch.int32: 2, torch.int64: 4, torch.uint8: 1,
       torch.int8: 0, torch.float64: 8}
_OPS = {"sum": 0, "prod": 1, "max": 2, "min": 3, "avg": 4}
DEFAULT_MIN_CHANNELS = 8
DEFAULT_MAX_CHANNELS = 16
_SEQ = collections.Counter()   # communicators created so far per group (ranks tuple): the unique-id store key
_LIVE = weakref.WeakSet()      # communicators to release at interpreter exit


@atexit.register
def _release_all():
    # local teardown only (ncclCommAbort frees this rank's resources without waiting for peers): a finalize at exit
    # could block on a peer that is already gone
    for c in list(_LIVE):
        c.destroy(abort=True)


def available():
    """(ok, where-or-why): whether librccl can be bound in this process."""
    rt = _native.runtime()
    msg = ctypes.c_char_p()
    ok = rt.dtfrt_rccl_available(ctypes.byref(msg)) == 0
    return ok, (msg.value or b"").decode()


def version():
    return int(_native.runtime().dtfrt_rccl_version())


def _check(rc, what):
    if rc != 0:
        s = _native.runtime().dtfrt_rccl_error_string(int(rc))
        raise RuntimeError(f"RCCL {what} failed: {rc} ({(s or b'').decode()})")


def _stream(t):
    return torch.cuda.current_stream(t.device).cuda_stream


class RcclCommunicator:
    """One RCCL communicator over the ranks of a torch.distributed group (collective construction: every rank of
    the group must create it at the same point)."""

    def __init__(self, group=None, device=None, min_channels=None, max_channels=None, name=None, self_check=True):
        import torch.distributed as dist
        ok, why = available()
        if not ok:
            raise RuntimeError(f"RCCL communicator unavailable: {why}")
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.device = device or torch.device("cuda", torch.cuda.current_device())
        self.min_channels = int(min_channels if min_channels is not None else DEFAULT_MIN_CHANNELS)
        self.max_channels = int(max_channels if max_channels is not None else DEFAULT_MAX_CHANNELS)
        if 0 < self.max_channels < self.min_channels:
            raise ValueError(f"max_channels {self.max_channels} < min_channels {self.min_channels}")
        # the store key names the group by its global ranks plus the number of communicators this process created for
        # that group before (every member creates them in the same order): disjoint groups whose rank 0s publish at
        # the same time can never read each other's id
        ranks = tuple(dist.get_process_group_ranks(group)) if group is not None else tuple(range(self.world))
        seq = _SEQ[ranks]
        _SEQ[ranks] += 1
        self.name = name or f"dtf{seq}"
        rt = _native.runtime()
        uid = ctypes.create_string_buffer(128)
        key = f"dtf_rccl/{'-'.join(map(str, ranks))}/{seq}/uid"
        store = dist.distributed_c10d._get_default_store()
        if self.rank == 0:
            _check(rt.dtfrt_rccl_unique_id(uid), "unique id")
            store.set(key, uid.raw)
        else:
            uid = ctypes.create_string_buffer(bytes(store.get(key)), 128)
        err = ctypes.c_int(0)
        with torch.cuda.device(self.device):
            self._h = rt.dtfrt_rccl_comm_init(uid, self.world, self.rank, self.min_channels, self.max_channels,
                                              self.name.encode(), ctypes.byref(err))
        if not self._h:
            _check(err.value or -1, "communicator init")
        _LIVE.add(self)
        if self_check:
            self._self_check()  # a collective: every rank has read the id once it returns
            if self.rank == 0:
                try:
                    store.delete_key(key)
                except (RuntimeError, AttributeError):  # a store without deletion: the key only lingers
                    pass

    def _self_check(self):
        t = torch.full((64,), float(self.rank + 1), device=self.device)
        self.all_reduce_(t)
        torch.cuda.synchronize(self.device)
        want = self.world * (self.world + 1) / 2
        if not bool((t == want).all()):
            self.destroy(abort=True)
            raise RuntimeError(f"RCCL communicator self-check failed: {t[0].item()} != {want}")

    # ---- collectives (stream-ordered on the current stream of the tensor's device)
    def all_reduce_(self, t, op="sum"):
        _check(_native.runtime().dtfrt_rccl_all_reduce(self._h, t.data_ptr(), t.data_ptr(), t.numel(), _DT[t.dtype],
                                                       _OPS[op], _stream(t)), "all_reduce")
        return t

    def reduce_scatter(self, inp, out, op="sum"):
        """out (n elements) = the reduced chunk `rank` of inp (world * n elements)."""
        if inp.numel() != out.numel() * self.world:
            raise ValueError("reduce_scatter: input must hold world * output elements")
        _check(_native.runtime().dtfrt_rccl_reduce_scatter(self._h, inp.data_ptr(), out.data_ptr(), out.numel(),
                                                           _DT[out.dtype], _OPS[op], _stream(out)), "reduce_scatter")
        return out

    def all_gather(self, inp, out):
        """out (world * n elements) = every rank's inp (n elements) in rank order."""
        if out.numel() != inp.numel() * self.world:
            raise ValueError("all_gather: output must hold world * input elements")
        _check(_native.runtime().dtfrt_rccl_all_gather(self._h, inp.data_ptr(), out.data_ptr(), inp.numel(),
                                                       _DT[inp.dtype], _stream(inp)), "all_gather")
        return out

    def broadcast_(self, t, root=0):
        _check(_native.runtime().dtfrt_rccl_broadcast(self._h, t.data_ptr(), t.data_ptr(), t.numel(), _DT[t.dtype],
                                                      root, _stream(t)), "broadcast")
        return t

    def send(self, t, peer):
        _check(_native.runtime().dtfrt_rccl_send(self._h, t.data_ptr(), t.numel(), _DT[t.dtype], peer, _stream(t)),
               "send")

    def recv(self, t, peer):
        _check(_native.runtime().dtfrt_rccl_recv(self._h, t.data_ptr(), t.numel(), _DT[t.dtype], peer, _stream(t)),
               "recv")
        return t

    def group_start(self):
        _check(_native.runtime().dtfrt_rccl_group_start(), "group_start")

    def group_end(self):
        _check(_native.runtime().dtfrt_rccl_group_end(), "group_end")

    # ---- state
    def info(self):
        n, r, calls, nbytes = ctypes.c_int(), ctypes.c_int(), ctypes.c_long(), ctypes.c_longlong()
        _check(_native.runtime().dtfrt_rccl_comm_info(self._h, ctypes.byref(n), ctypes.byref(r), ctypes.byref(calls),
                                                      ctypes.byref(nbytes)), "comm info")
        return {"nranks": n.value, "rank": r.value, "calls": calls.value, "bytes": nbytes.value,
                "min_channels": self.min_channels, "max_channels": self.max_channels}

    def async_error(self):
        return int(_native.runtime().dtfrt_rccl_async_error(self._h))

    def destroy(self, abort=False):
        """Release the communicator (abort=False: finalize = wait for its outstanding collectives, which needs the
        peers alive; abort=True: local teardown). Idempotent."""
        h, self._h = getattr(self, "_h", None), None
        _LIVE.discard(self)
        if h:
            _native.runtime().dtfrt_rccl_comm_destroy(h, int(bool(abort)))

    def __del__(self):
        try:
            self.destroy(abort=True)
        except Exception:
            pass


def wanted(implementation=None):
    """Whether the bucketer should drive the native communicator: CommunicationImplementation.NCCL asks for it,
    RING for torch.distributed's process group, AUTO (None) follows DTF_COMM ("native" / "torch", default native on
    GPU process groups)."""
    impl = getattr(implementation, "value", implementation)
    if impl is not None:
        impl = str(impl).lower()
        if impl in ("nccl", "rccl", "native"):
            return True
        if impl in ("ring", "torch"):
            return False
    return os.environ.get("DTF_COMM", "native").lower() == "native"
