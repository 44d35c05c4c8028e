"""Device context: where new variables and tensors are placed.

TF's device placer (reference trainer/task.py:124-127 scopes graph building
under ``replica_device_setter``) becomes a small stack of torch devices. The
default is the process's local GPU (one process per GPU, ``LOCAL_RANK``) or the
CPU when no GPU is visible.
"""
from __future__ import annotations

import contextlib
import os
import re
import threading

import torch

_tls = threading.local()


def _stack():
    s = getattr(_tls, "stack", None)
    if s is None:
        s = []
        _tls.stack = s
    return s


def local_ordinal(default=0) -> int:
    """This process's GPU ordinal among the visible devices: DTF_DEVICE_ORDINAL (set per task by cli.launch, which
    keeps every GPU visible so PS tasks and trainers can map each other's memory), else LOCAL_RANK (torchrun), else
    `default`."""
    return int(os.environ.get("DTF_DEVICE_ORDINAL", os.environ.get("LOCAL_RANK", str(default))))


def default_device() -> torch.device:
    """The process's own GPU (local_ordinal), or the CPU when no GPU is visible."""
    if torch.cuda.is_available():
        return torch.device("cuda", local_ordinal() % max(1, torch.cuda.device_count()))
    return torch.device("cpu")


def bind_device(dev) -> torch.device:
    """Make `dev` the process's current HIP device. Every kernel wrapper issues on the CURRENT device's stream
    (ops._util.stream), so a task whose GPU is not ordinal 0 must bind it before its first op — otherwise a copy
    issued on cuda:k's stream and a kernel issued on cuda:0's stream are unordered."""
    dev = parse_device(dev)
    if dev.type == "cuda":
        torch.cuda.set_device(dev)
    return dev


def current_device() -> torch.device:
    s = _stack()
    return s[-1] if s else default_device()


def parse_device(spec) -> torch.device:
    """'/GPU:1', '/job:worker/task:0/device:CPU:0', 'cpu', 'cuda:0' or torch.device -> torch.device."""
    if isinstance(spec, torch.device):
        return spec
    s = str(spec)
    m = re.search(r"(GPU|CPU|gpu|cpu|cuda)(?::(\d+))?$", s)
    if not m:
        return torch.device(s)
    kind, idx = m.group(1).lower(), int(m.group(2) or 0)
    if kind in ("gpu", "cuda"):
        return torch.device("cuda", idx)
    return torch.device("cpu")


@contextlib.contextmanager
def device(spec):
    d = parse_device(spec)
    _stack().append(d)
    try:
        if d.type == "cuda":
            with torch.cuda.device(d):
                yield d
        else:
            yield d
    finally:
        _stack().pop()


def list_physical_devices(kind=None):
    out = []
    if kind in (None, "CPU"):
        out.append("/physical_device:CPU:0")
    if kind in (None, "GPU") and torch.cuda.is_available():
        out += [f"/physical_device:GPU:{i}" for i in range(torch.cuda.device_count())]
    return out
