"""Tracing / profiling (SURVEY §5 "Tracing / profiling").

The reference only has wall-clock ``datetime`` deltas (reference trainer/task.py:39,100-102,250-252).
Here:
* ``range(name)`` / ``mark(msg)``: roctx ranges and markers (libroctx64, loaded with ctypes) that show
  up in ``rocprofv3 --marker-trace`` timelines; no-ops when the library or ``DTF_ROCTX=0``;
* ``PhaseTimer``: hipEvent-based per-phase device time of a training step (forward / backward /
  all-reduce / optimizer) without host synchronisation inside the step — read it when you want;
* ``StepStats``: host-side step-time and throughput meter (images/sec, tokens/sec, global_step/sec)
  that also writes TensorBoard scalars like the Supervisor's step counter thread
  (``global_step/sec``, reference trainer/task.py:215-223 [TF-RT]).
``Model.train_step`` brackets its phases with ``phase(...)`` so enabling roctx (``enable()``) or a
PhaseTimer requires no code changes in user loops.
"""
from __future__ import annotations

import contextlib
import ctypes
import os
import time

import torch

_lib = None
_enabled = os.environ.get("DTF_ROCTX", "0") == "1"
_timer = None  # active PhaseTimer


def _roctx():
    global _lib
    if _lib is None:
        _lib = False
        for name in ("libroctx64.so", "libroctx64.so.4", "/opt/rocm/lib/libroctx64.so"):
            try:
                lib = ctypes.CDLL(name)
                lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
                lib.roctxRangePushA.restype = ctypes.c_int
                lib.roctxRangePop.restype = ctypes.c_int
                lib.roctxMarkA.argtypes = [ctypes.c_char_p]
                _lib = lib
                break
            except OSError:
                continue
    return _lib or None


def enable(on=True):
    """Turn roctx ranges on/off process-wide (equivalent to DTF_ROCTX=1)."""
    global _enabled
    _enabled = bool(on)


def available():
    return _roctx() is not None


@contextlib.contextmanager
def range(name):  # noqa: A001  (mirrors roctx naming)
    lib = _roctx() if _enabled else None
    if lib is not None:
        lib.roctxRangePushA(name.encode())
    try:
        yield
    finally:
        if lib is not None:
            lib.roctxRangePop()


def mark(msg):
    lib = _roctx() if _enabled else None
    if lib is not None:
        lib.roctxMarkA(str(msg).encode())


class PhaseTimer:
    """Per-phase device time via hipEvents recorded on the current stream.

    with PhaseTimer() as pt:
        for _ in range(n): model.train_step(batch)
    pt.summary() -> {"forward": ms/step, "backward": ..., ...}
    """

    def __init__(self):
        self.events = []  # (phase, start_event, end_event)
        self.steps = 0

    def __enter__(self):
        global _timer
        self._prev, _timer = _timer, self
        return self

    def __exit__(self, *exc):
        global _timer
        _timer = self._prev

    def begin(self, phase):
        if not torch.cuda.is_available():
            return None
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        self.events.append((phase, s, e))
        return e

    def summary(self):
        torch.cuda.synchronize()
        tot = {}
        for phase, s, e in self.events:
            tot[phase] = tot.get(phase, 0.0) + s.elapsed_time(e)
        n = max(1, self.steps)
        return {k: v / n for k, v in tot.items()}


@contextlib.contextmanager
def phase(name):
    """One training-step phase: a roctx range plus, under a PhaseTimer, a pair of hipEvents."""
    t = _timer
    end = t.begin(name) if t is not None else None
    with range(name):
        yield
    if end is not None:
        end.record()
        if name == "optimizer":
            t.steps += 1


class StepStats:
    """Host step timer + throughput meter; optional TensorBoard scalars (``global_step/sec``, items/sec)."""

    def __init__(self, items_per_step=1, unit="items/sec", writer=None, every=100):
        self.items_per_step = items_per_step
        self.unit = unit
        self.writer = writer
        self.every = every
        self.t_last = None
        self.n = 0
        self.history = []

    def step(self, global_step=None):
        now = time.perf_counter()
        if self.t_last is None:
            self.t_last = now
            return None
        self.n += 1
        if self.n % self.every:
            return None
        dt = (now - self.t_last) / self.every
        self.t_last = now
        rec = {"sec_per_step": dt, "global_step/sec": 1.0 / dt, self.unit: self.items_per_step / dt}
        self.history.append(rec)
        if self.writer is not None and global_step is not None:
            self.writer.scalar("global_step/sec", rec["global_step/sec"], global_step)
            self.writer.scalar(self.unit, rec[self.unit], global_step)
        return rec
