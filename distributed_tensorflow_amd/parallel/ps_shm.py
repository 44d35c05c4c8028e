"""Intra-node parameter-server data plane: direct copies into PS-owned memory + a shared-memory mailbox.

The reference pulls every variable from and pushes every gradient to the PS tasks through TF's gRPC Send/Recv
rendezvous on each step (reference trainer/task.py:124-127, 236 [TF-RT]). On one MI355X node the
bytes should move once, GPU to GPU over xGMI, with no host staging and no RCCL communicator per (ps, trainer) pair
(round 1's design kept one blocked RCCL recv per trainer spinning on each PS GPU). Here:

* Each PS task owns, in its own device's memory, its variable shard (the optimizer arena: contiguous, in the
  trainers' arena order), its optimizer slots, and ONE GRADIENT INBOX PER TRAINER. GPU PS: HBM exported with HIP
  IPC handles (csrc/kernels/ipc.hip); CPU PS: named POSIX shared memory (csrc/runtime/ps_mailbox.cc), with a
  published copy of the parameters refreshed after every apply.
* A trainer's gradient push is one device-to-device copy of its shard slice into its inbox (hipMemcpyAsync into
  the IPC-mapped peer memory: an xGMI transfer issued on the trainer's own stream), then a mailbox post; its pull
  is one copy out of the PS's parameter buffer. Shards are contiguous slices of the trainer's arena (the strategy
  lays the arena out grouped by PS, ParameterServerStrategy.order_variables), so there is no gather / index_select.
* The control plane is the native mailbox (one 64-B slot per trainer, futex doorbells): ONE serve loop per PS
  applies requests in arrival order with the fused optimizer kernel — no per-trainer threads, no host sync per
  request beyond the apply itself, no GPU spin-waits occupying hardware queues.
Semantics are the reference's asynchronous (Hogwild) PS training: every push is applied whole, in arrival order;
pulls read the live parameters without a lock (TF's use_locking=False apply ops, trainer/task.py:138).
"""
from __future__ import annotations

import ctypes
import json
import os
import secrets

import numpy as np
import torch

from .. import _native
from .._runtime_sigs import err

OP_PUSH, OP_ASSIGN, OP_DONE, OP_PUSH_ASYNC = 1, 2, 3, 4


def _rt():
    return _native.runtime()


def _host_tensor(ptr, numel):
    buf = (ctypes.c_float * numel).from_address(ptr)
    return torch.from_numpy(np.ctypeslib.as_array(buf))


class _Region:
    """Memory a PS shares with its trainers: a local tensor on the PS side, a descriptor for the trainers."""

    def __init__(self, numel, device, name):
        self.numel, self.device, self.name = int(numel), device, name
        self._shm = None
        if device.type == "cuda":
            self.tensor = torch.zeros(max(1, self.numel), dtype=torch.float32, device=device)
            handle = ctypes.create_string_buffer(64)
            off = ctypes.c_long()
            _native.call("dtf_ipc_export", self.tensor.data_ptr(), handle, ctypes.addressof(off))
            self.desc = {"kind": "hip", "handle": handle.raw.hex(), "offset": off.value, "numel": self.numel,
                         "device": device.index}
        else:
            nbytes = max(4, self.numel * 4)
            p = _rt().dtfrt_shmem_create(name.encode(), nbytes)
            if not p:
                raise OSError(err(_rt()))
            self._shm = (p, nbytes)
            self.tensor = _host_tensor(p, max(1, self.numel))
            self.tensor.zero_()
            self.desc = {"kind": "host", "name": name, "numel": self.numel}

    def close(self):
        if self._shm is not None:
            _rt().dtfrt_shmem_close(self._shm[0], self._shm[1], self.name.encode(), 1)
            self._shm = None


_IPC_MAPS = {}  # (handle hex, local device index) -> [mapped base, open count]


def _ipc_open(handle_hex, device):
    """Map a peer allocation once per process: several exported PS regions (inbox, parameters, slots) can live in
    ONE caching-allocator segment and so carry the same IPC handle; each distinct handle is opened once and
    reference-counted (repeated hipIpcOpenMemHandle / close of one handle is driver-dependent)."""
    key = (handle_hex, device.index)
    ent = _IPC_MAPS.get(key)
    if ent is None:
        base = ctypes.c_void_p()
        _native.call("dtf_ipc_open", bytes.fromhex(handle_hex), ctypes.addressof(base))
        ent = _IPC_MAPS[key] = [base.value, 0]
    ent[1] += 1
    return ent[0]


def _ipc_release(handle_hex, device):
    key = (handle_hex, device.index)
    ent = _IPC_MAPS.get(key)
    if ent is None:
        return
    ent[1] -= 1
    if ent[1] <= 0:
        _native.call("dtf_ipc_close", ent[0])
        del _IPC_MAPS[key]


class _Remote:
    """A trainer's mapping of one PS region: copy_in / copy_out between a local f32 slice and the region."""

    def __init__(self, desc, device):
        self.desc, self.numel = desc, int(desc["numel"])
        self.device = device
        self._shm = None
        self._mapped = False
        if desc["kind"] == "hip":
            if device.type != "cuda":
                raise RuntimeError("the PS shard lives in GPU memory but this task has no GPU")
            self._base = _ipc_open(desc["handle"], device)
            self._mapped = True
            self.ptr = self._base + int(desc["offset"])
            self.tensor = None
        else:
            nbytes = max(4, self.numel * 4)
            p = _rt().dtfrt_shmem_open(desc["name"].encode(), nbytes, 60000)
            if not p:
                raise OSError(err(_rt()))
            self._shm = (p, nbytes)
            self.tensor = _host_tensor(p, max(1, self.numel))
            self.ptr = p

    def copy_in(self, src, offset=0):
        """region[offset:offset+n] <- src (f32 contiguous), stream-ordered on the caller's stream (GPU)."""
        n = src.numel()
        if self.tensor is not None:
            self.tensor[offset:offset + n].copy_(src.detach().reshape(-1).cpu() if src.is_cuda else src.reshape(-1))
        else:
            from ..ops._util import stream
            _native.call("dtf_memcpy_async", self.ptr + 4 * offset, src.data_ptr(), 4 * n, stream(src.device))

    def copy_out(self, dst, offset=0):
        """dst <- region[offset:offset+n]."""
        n = dst.numel()
        if self.tensor is not None:
            dst.reshape(-1).copy_(self.tensor[offset:offset + n])
        else:
            from ..ops._util import stream
            _native.call("dtf_memcpy_async", dst.data_ptr(), self.ptr + 4 * offset, 4 * n, stream(dst.device))

    def close(self):
        if self._shm is not None:
            _rt().dtfrt_shmem_close(self._shm[0], self._shm[1], None, 0)
            self._shm = None
        elif self._mapped:
            _ipc_release(self.desc["handle"], self.device)
            self._mapped = False


def _sync(device):
    """Host waits for the work issued so far on `device`'s current stream (one recorded event, not the device)."""
    if device.type == "cuda":
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(device))
        ev.synchronize()


# ---------------------------------------------------------------------------------------------- PS side
class ShmPSServer:
    """The PS task's serve loop over the mailbox (one thread, requests applied in arrival order)."""

    def __init__(self, ps, kv, num_trainers, timeout_s=900):
        self.ps, self.kv, self.T = ps, kv, num_trainers
        self.dev = ps.device
        tag = secrets.token_hex(4)
        base = f"dtf{os.getpid()}_{ps.index}_{tag}"
        n = int(ps.arena.numel) if ps.arena is not None else 0
        self.params = None if ps.arena is None or self.dev.type == "cuda" else _Region(n, self.dev, base + "_p")
        self.inboxes = [_Region(n, self.dev, f"{base}_in{t}") for t in range(num_trainers)]
        self.slots = []
        if ps.arena is not None and self.dev.type != "cuda":
            self.slots = [_Region(n, self.dev, f"{base}_s{k}") for k, _ in enumerate(ps.opt.slot_specs())]
        self.mbox = _rt().dtfrt_mbox_create(f"{base}_mb".encode(), max(1, num_trainers))
        if not self.mbox:
            raise OSError(err(_rt()))
        self.timeout_s = timeout_s
        desc = {"numel": n, "mbox": f"{base}_mb", "inboxes": [r.desc for r in self.inboxes]}
        if ps.arena is not None and self.dev.type == "cuda":
            # the live arena and slot arenas are shared directly (no publish copy)
            desc["params"] = _export(ps.arena.flat, self.dev)
            desc["slots"] = [_export(ps.arena.slots[nm], self.dev) for nm, _ in ps.opt.slot_specs()]
        elif ps.arena is not None:
            self._publish(slots=True)
            desc["params"] = self.params.desc
            desc["slots"] = [r.desc for r in self.slots]
        kv.set(f"ps/{ps.index}/shm", json.dumps(desc))

    def _publish(self, slots=False):
        if self.params is None:
            return
        self.params.tensor[:self.params.numel].copy_(self.ps.arena.flat)
        if slots:
            for r, (nm, _) in zip(self.slots, self.ps.opt.slot_specs()):
                r.tensor[:r.numel].copy_(self.ps.arena.slots[nm])

    def serve(self, forever=False):
        lib = _rt()
        slot, op, seq, arg = ctypes.c_int(), ctypes.c_int(), ctypes.c_int64(), ctypes.c_uint64()
        finished = set()
        # an apply that fails AFTER its early acknowledgement (OP_PUSH_ASYNC) cannot fail that request any more: the
        # error is kept per trainer and returned as the status of the trainer's NEXT request, which the trainer's
        # wait (wait_pending / the next push, pull or done) raises — a gradient is never dropped silently
        deferred = {}
        while forever or len(finished) < self.T:
            got = lib.dtfrt_mbox_next(self.mbox, 200, ctypes.addressof(slot), ctypes.addressof(op),
                                      ctypes.addressof(seq), ctypes.addressof(arg))
            if not got:
                if not forever and self.kv.wait_ge("done", self.T, timeout_s=0):
                    break
                continue
            t, status, acked = slot.value, 0, [False]
            if t in deferred:
                lib.dtfrt_mbox_complete(self.mbox, t, seq.value, deferred.pop(t))
                if op.value == OP_DONE:
                    finished.add(t)
                continue

            def ack_early(t=t, s=seq.value):
                # the inbox has been consumed (the gradient copy landed): the trainer may refill it while the update
                # itself is still running — an OP_PUSH_ASYNC trainer does not wait for the apply (bounded staleness 1)
                lib.dtfrt_mbox_complete(self.mbox, t, s, 0)
                acked[0] = True
            try:
                if op.value == OP_DONE:
                    finished.add(t)
                elif self.ps.arena is not None:
                    inbox = self.inboxes[t].tensor[:self.ps.arena.numel]
                    early = op.value == OP_PUSH_ASYNC
                    self.ps.apply_flat(inbox, assign=(op.value == OP_ASSIGN), consumed=ack_early if early else None)
                    self._publish(slots=(op.value == OP_ASSIGN or self.ps.applies % self.ps.slot_sync_every == 0))
                    if not early:
                        _sync(self.dev)  # OP_PUSH / OP_ASSIGN: the parameters a trainer pulls next are the updated ones
            except Exception as e:  # report to the pushing trainer instead of dying silently
                print(f"[ps{self.ps.index}] request {op.value} from trainer {t} failed: {e}", flush=True)
                status = -7
                if acked[0]:
                    deferred[t] = status
            if not acked[0]:
                lib.dtfrt_mbox_complete(self.mbox, t, seq.value, status)
        self._publish(slots=True)

    def close(self):
        if self.mbox:
            _rt().dtfrt_mbox_close(self.mbox, 1)
            self.mbox = None
        for r in self.inboxes + self.slots + ([self.params] if self.params else []):
            r.close()


def _export(t, dev):
    handle = ctypes.create_string_buffer(64)
    off = ctypes.c_long()
    _native.call("dtf_ipc_export", t.data_ptr(), handle, ctypes.addressof(off))
    return {"kind": "hip", "handle": handle.raw.hex(), "offset": off.value, "numel": int(t.numel()),
            "device": dev.index}


# ---------------------------------------------------------------------------------------------- trainer side
class ShmPSClient:
    """Trainer side: maps every PS's buffers and mailbox; push / assign / pull per contiguous shard slice.

    segments[p]: list of (arena_offset, shard_offset, numel) runs of the trainer's arena that belong to PS p (one
    run when the arena is grouped by PS)."""

    def __init__(self, kv, num_ps, trainer_index, device, segments, timeout_s=900, staleness=0):
        self.kv, self.P, self.t, self.dev = kv, num_ps, trainer_index, device
        self.segments = segments
        # staleness 0: a push returns once every PS applied it (the next pull sees this trainer's update, TF's
        # sess.run(train_op) semantics); 1: a push returns once its bytes are in the inboxes — the PS acknowledges
        # as soon as it has consumed them, and the trainer only waits for that acknowledgement before it refills the
        # inbox on its NEXT push (its next pull may miss its own latest update: Hogwild with staleness <= 1)
        self.staleness = int(staleness)
        self._pending = []
        self.timeout_ms = int(timeout_s * 1000)
        self.desc = [kv.get_json(f"ps/{p}/shm", timeout_s=timeout_s) for p in range(num_ps)]
        self.inbox = [_Remote(d["inboxes"][trainer_index], device) for d in self.desc]
        self.params = [_Remote(d["params"], device) if "params" in d else None for d in self.desc]
        self.slots = [[_Remote(s, device) for s in d.get("slots", [])] for d in self.desc]
        lib = _rt()
        self.mbox = []
        for d in self.desc:
            h = lib.dtfrt_mbox_open(d["mbox"].encode(), self.timeout_ms)
            if not h:
                raise ConnectionError(err(lib))
            self.mbox.append(h)

    def _wait(self, seqs, op):
        lib = _rt()
        for p, s in seqs:
            st = lib.dtfrt_mbox_wait(self.mbox[p], self.t, s, self.timeout_ms)
            if st != 0:
                raise ConnectionError(f"ps{p}: request {op} failed ({st}): {err(lib)}")

    def _post_all(self, op, ps_list, wait=True):
        lib = _rt()
        seqs = [(p, lib.dtfrt_mbox_post(self.mbox[p], self.t, op, 0)) for p in ps_list]
        if wait:
            self._wait(seqs, op)
        else:
            self._pending = seqs

    def wait_pending(self):
        """Block until the PS tasks consumed this trainer's previous push (its inboxes may be refilled)."""
        if self._pending:
            seqs, self._pending = self._pending, []
            self._wait(seqs, OP_PUSH_ASYNC)

    def _ps_list(self):
        return [p for p in range(self.P) if self.segments[p]]

    def copy_range(self, src_flat, lo, hi):
        """Issue the inbox copies of the arena elements [lo, hi) on the current stream (one bucket of a push)."""
        for p in self._ps_list():
            for ao, so, n in self.segments[p]:
                a, b = max(ao, lo), min(ao + n, hi)
                if a < b:
                    self.inbox[p].copy_in(src_flat[a:b], so + (a - ao))

    def post_push(self):
        """Tell every PS that this trainer's gradient is in its inbox (the copies must have landed)."""
        if self.staleness > 0:
            self._post_all(OP_PUSH_ASYNC, self._ps_list(), wait=False)
        else:
            self._post_all(OP_PUSH, self._ps_list())

    def _send(self, src_flat, op):
        self.wait_pending()
        ps_list = self._ps_list()
        for p in ps_list:
            for ao, so, n in self.segments[p]:
                self.inbox[p].copy_in(src_flat[ao:ao + n], so)
        _sync(self.dev)  # the inbox bytes have landed before the PS is told
        if op == OP_PUSH:
            self.post_push()
        else:
            self._post_all(op, ps_list)

    def push(self, grad_flat):
        self._send(grad_flat, OP_PUSH)

    def assign(self, flat):
        self._send(flat, OP_ASSIGN)

    def pull(self, flat):
        """flat <- the live PS parameters. GPU PS: peer copies on the current stream (stream-ordered before every
        later kernel: no host wait); CPU PS: host copies."""
        for p in range(self.P):
            for ao, so, n in self.segments[p]:
                self.params[p].copy_out(flat[ao:ao + n], so)

    def pull_slots(self, nslots, like):
        out = [torch.zeros_like(like) for _ in range(nslots)]
        for p in range(self.P):
            for k in range(nslots):
                for ao, so, n in self.segments[p]:
                    self.slots[p][k].copy_out(out[k][ao:ao + n], so)
        return out

    def done(self):
        self.wait_pending()
        self._post_all(OP_DONE, list(range(self.P)))

    def close(self):
        lib = _rt()
        for h in self.mbox:
            lib.dtfrt_mbox_close(h, 0)
        self.mbox = []
        for r in self.inbox + [x for x in self.params if x is not None] + [s for ss in self.slots for s in ss]:
            r.close()
