"""One-shot peer-to-peer all-reduce of small gradient buckets over IPC-mapped HBM (csrc/kernels/p2p_allreduce.hip).

RCCL's ring/tree all-reduce pays a fixed latency per collective; for the small buckets at the tail of a backward
pass (the ones whose reduction is exposed after the last gradient lands) every rank instead reads the bucket
straight from each peer's gradient arena over xGMI — all 7 links of an MI355X at once — and sums it in rank order
in registers ("custom one-shot P2P all-reduce over IPC-mapped HBM for small buckets"). The
result is bitwise identical on every rank and equal to the ordered f32 sum x0 + x1 + ... + x_{W-1}.

Setup (collective, once per gradient arena): every rank exports its arena gradient, a same-sized f32 scratch and a
flag array with HIP IPC handles (dtf_ipc_export); the handles travel through the process group
(all_gather_object: gloo or RCCL) and every rank maps its peers' buffers. Requirements: all ranks on one node
(same hostname), at most 8 ranks, CUDA tensors. A call launches ONE kernel on the current stream (stream-ordered
after the kernels that produced the bucket, before the ones that consume it) with a host-side epoch; every rank
must issue the same calls in the same order (the bucketer's bucket order guarantees it). Not used under hipGraph
capture (the epoch is a kernel argument). The bucketer issues the kernel on the communication stream (which waits for
the main and weight-gradient streams), so a spin waiting for a slow peer holds no weight-gradient GEMM behind it.
Opt-in: DTF_P2P=1 (see available()).
"""
from __future__ import annotations

import ctypes
import os
import socket

import torch
import torch.distributed as dist

from .. import _native

MAX_RANKS = 8
NBLK = 64  # blocks per rank and call
# buckets up to this size (bytes, f32) take the P2P path when it is available (DTF_P2P_MAX_KB; 0 disables)
MAX_BYTES = int(float(os.environ.get("DTF_P2P_MAX_KB", "4096")) * 1024)
# a spinning block gives up after this long (a peer rank far behind, e.g. writing a checkpoint, is waited for)
TIMEOUT_MS = int(os.environ.get("DTF_P2P_TIMEOUT_MS", "300000"))
PROBE = 4096 + 3  # floats of the set-up self-test (exercises the float4 body and the scalar tail)


def _export(t):
    handle = ctypes.create_string_buffer(64)
    off = ctypes.c_long()
    _native.call("dtf_ipc_export", t.data_ptr(), handle, ctypes.addressof(off))
    return handle.raw.hex(), off.value


def _open(handle_hex, offset):
    ptr = ctypes.c_void_p()
    _native.call("dtf_ipc_open", bytes.fromhex(handle_hex), ctypes.addressof(ptr))
    return ptr.value, ptr.value + offset


class P2PAllReducer:
    """Bucket all-reduce over IPC-mapped peer gradient arenas (see module docstring)."""

    def __init__(self, grad, group=None, spans=None):
        """spans: the [lo, hi) arena ranges that will be reduced here (the P2P-eligible buckets); the kernel's f32
        scratch covers only those (default: the whole arena)."""
        if grad.device.type != "cuda" or grad.dtype != torch.float32:
            raise ValueError("P2P all-reduce needs an f32 CUDA gradient arena")
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        if self.world > MAX_RANKS:
            raise ValueError(f"P2P all-reduce supports at most {MAX_RANKS} ranks")
        self.grad = grad
        dev = grad.device
        spans = [(0, grad.numel())] if spans is None else sorted(spans)
        self._soff = {}
        tot = 0
        for lo, hi in spans:
            self._soff[(lo, hi)] = tot
            tot += -(-(hi - lo) // 4) * 4  # 16-B aligned slices
        self.red = torch.empty(max(tot, 4), dtype=torch.float32, device=dev)
        self.flags = torch.zeros(2 * NBLK * MAX_RANKS, dtype=torch.int32, device=dev)
        self.err = torch.zeros(1, dtype=torch.int32, device=dev)
        torch.cuda.synchronize(dev)
        mine = {"host": socket.gethostname(), "grad": _export(grad), "flags": _export(self.flags)}
        allv = [None] * self.world
        dist.all_gather_object(allv, mine, group=group)
        if len({v["host"] for v in allv}) != 1:
            raise RuntimeError("P2P all-reduce needs every rank on one node")
        self._mapped = []
        self.grad_ptr = [0] * self.world
        self.flag_ptr = [0] * self.world
        for p, v in enumerate(allv):
            if p == self.rank:
                self.grad_ptr[p], self.flag_ptr[p] = grad.data_ptr(), self.flags.data_ptr()
                continue
            base, g = _open(*v["grad"])
            self._mapped.append(base)
            fbase, f = _open(*v["flags"])
            self._mapped.append(fbase)
            self.grad_ptr[p], self.flag_ptr[p] = g, f
        self.epoch = 0
        self.calls = 0
        self._err_host = torch.zeros(1, dtype=torch.int32).pin_memory()
        self._err_ev = None
        if not self._selftest(allv):
            self.close()
            raise RuntimeError("P2P all-reduce self-test failed (peer memory not reachable or wrong sums)")

    def _selftest(self, allv):
        """One call over a small probe buffer of every rank (value rank + 1) with a short timeout: every rank must
        hold the exact sum. All ranks agree on the outcome (a failure anywhere disables the path everywhere)."""
        dev = self.grad.device
        probe = torch.full((PROBE,), float(self.rank + 1), dtype=torch.float32, device=dev)
        pred = torch.empty_like(probe)
        torch.cuda.synchronize(dev)
        mine = _export(probe)
        allp = [None] * self.world
        dist.all_gather_object(allp, mine, group=self.group)
        ptrs, opened = [], []
        ok = True
        try:
            for p, v in enumerate(allp):
                if p == self.rank:
                    ptrs.append(probe.data_ptr())
                    continue
                base, q = _open(*v)
                opened.append(base)
                ptrs.append(q)
            self.epoch += 1
            srcs = (ctypes.c_void_p * self.world)(*ptrs)
            flags = (ctypes.c_void_p * self.world)(*self.flag_ptr)
            from ..ops._util import stream
            _native.call("dtf_p2p_allreduce_f32", probe.data_ptr(), srcs, pred.data_ptr(), self.flags.data_ptr(),
                         flags, PROBE, self.world, self.rank, self.epoch, 1, 5000, self.err.data_ptr(), stream(dev))
            torch.cuda.synchronize(dev)
            want = float(self.world * (self.world + 1) // 2)
            ok = int(self.err.item()) == 0 and bool((probe == want).all().item())
        except (RuntimeError, OSError):
            ok = False
        finally:
            torch.cuda.synchronize(dev)
            dist.barrier(group=self.group)  # no peer reads this rank's probe any more
            for base in opened:
                _native.call("dtf_ipc_close", base)
        self.err.zero_()
        flag = torch.tensor([1 if ok else 0], dtype=torch.int64, device=dev if dist.get_backend(self.group) == "nccl"
                            else "cpu")
        dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=self.group)
        return bool(flag.item())

    def poll(self):
        """Raise if a spin of an EARLIER step timed out (read back asynchronously: no device sync)."""
        if self._err_ev is not None and self._err_ev.query():
            if int(self._err_host.item()):
                raise RuntimeError("P2P all-reduce timed out waiting for a peer rank (the step's sums are wrong)")
            self._err_ev = None
        if self._err_ev is None and not torch.cuda.is_current_stream_capturing():
            self._err_host.copy_(self.err, non_blocking=True)
            self._err_ev = torch.cuda.Event()
            self._err_ev.record()

    def all_reduce_(self, lo, hi, timeout_ms=None):
        """Sum grad[lo:hi] over the ranks in place (on the current stream). [lo, hi) must be one of the spans given
        at construction, or lie inside the whole-arena default span."""
        n = hi - lo
        if n <= 0:
            return
        soff = self._soff.get((lo, hi))
        if soff is None:
            whole = self._soff.get((0, self.grad.numel()))
            if whole is None:
                raise ValueError(f"P2P all-reduce of [{lo}, {hi}): not a span given at construction")
            soff = lo
        self.epoch += 1
        self.calls += 1
        srcs = (ctypes.c_void_p * self.world)(*[p + 4 * lo for p in self.grad_ptr])
        flags = (ctypes.c_void_p * self.world)(*self.flag_ptr)
        nblk = max(1, min(NBLK, -(-n // (256 * 4 * 4))))  # >= 4 float4 per thread
        from ..ops._util import stream
        _native.call("dtf_p2p_allreduce_f32", self.grad.data_ptr() + 4 * lo, srcs, self.red.data_ptr() + 4 * soff,
                     self.flags.data_ptr(), flags, n, self.world, self.rank, self.epoch, nblk,
                     TIMEOUT_MS if timeout_ms is None else int(timeout_ms), self.err.data_ptr(),
                     stream(self.grad.device))

    def check(self):
        """Raise if any call timed out waiting for a peer (synchronises the device)."""
        if int(self.err.item()):
            raise RuntimeError("P2P all-reduce timed out waiting for a peer rank")

    def close(self):
        for base in self._mapped:
            _native.call("dtf_ipc_close", base)
        self._mapped = []


def available(grad, group=None):
    """Whether the P2P path can be used for this arena (CUDA f32, <= 8 ranks; node locality is checked at setup).
    Opt-in (DTF_P2P=1) until a cross-GPU run has validated it: every test so far shares one GPU between the ranks
    (ADVICE r4)."""
    return (MAX_BYTES > 0 and grad.is_cuda and grad.dtype == torch.float32 and dist.is_initialized()
            and 1 < dist.get_world_size(group) <= MAX_RANKS and os.environ.get("DTF_P2P", "0") == "1")
