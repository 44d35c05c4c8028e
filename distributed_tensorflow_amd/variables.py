"""Variables and flat parameter arenas.

``Variable`` mirrors the tf.Variable surface the reference uses (``weight``,
``bias`` and the untrainable ``global_step`` of reference trainer/task.py:66-68,
134-136: a name, ``trainable``, ``assign``/``assign_add``, ``numpy``) and is a
``torch.nn.Parameter`` underneath so it flows straight into autograd and the
HIP ops.

``ParamArena`` is the MI355X-first storage layout for a set of variables: one
contiguous f32 master buffer, one contiguous f32 gradient buffer, a bf16
compute-copy buffer and one buffer per optimizer slot. Each variable becomes a
view into the arena, so
  * the optimizer update is ONE streaming kernel over the whole model,
  * gradient all-reduce buckets are plain slices of the gradient arena (no
    pack/unpack copies — SURVEY §2.6 K18 becomes a no-op),
  * checkpoints and PS shards are contiguous byte ranges.
Sizes are padded to 64 elements so every view is 256-B aligned (16-B vector
loads in the kernels, 128-B cache lines).
"""
from __future__ import annotations

import itertools
import threading

import numpy as np
import torch

_uid = itertools.count()
_name_lock = threading.Lock()
_name_counts: dict = {}


def unique_name(base: str) -> str:
    with _name_lock:
        n = _name_counts.get(base, 0)
        _name_counts[base] = n + 1
    return base if n == 0 else f"{base}_{n}"


def reset_names():
    with _name_lock:
        _name_counts.clear()


class Variable(torch.nn.Parameter):
    """A named, optionally trainable tensor variable (tf.Variable analogue)."""

    def __new__(cls, initial_value=0.0, trainable=True, name=None, dtype=None, device=None):
        if callable(initial_value):
            initial_value = initial_value()
        t = torch.as_tensor(np.asarray(initial_value) if not isinstance(initial_value, torch.Tensor)
                            else initial_value)
        if dtype is not None:
            t = t.to(dtype)
        elif t.is_floating_point() and t.dtype == torch.float64:
            t = t.to(torch.float32)
        if device is not None:
            t = t.to(device)
        requires_grad = bool(trainable) and t.is_floating_point()
        obj = torch.Tensor._make_subclass(cls, t.detach().clone(), requires_grad)
        obj._dtf_name = name or unique_name("Variable")
        obj._dtf_trainable = bool(trainable)
        return obj

    # torch.nn.Parameter has a custom __deepcopy__/__reduce_ex__; keep ours simple
    def __deepcopy__(self, memo):
        v = Variable(self.detach().clone(), trainable=self._dtf_trainable, name=self._dtf_name)
        memo[id(self)] = v
        return v

    def __reduce_ex__(self, proto):
        return (_rebuild_variable, (self.detach().cpu(), self._dtf_trainable, self._dtf_name))

    @property
    def name(self):
        return self._dtf_name

    @property
    def trainable(self):
        return self._dtf_trainable

    def assign(self, value):
        with torch.no_grad():
            self.copy_(torch.as_tensor(value, dtype=self.dtype).to(self.device))
        _touch(self)
        return self

    def assign_add(self, value):
        with torch.no_grad():
            self.add_(torch.as_tensor(value, dtype=self.dtype).to(self.device))
        _touch(self)
        return self

    def assign_sub(self, value):
        with torch.no_grad():
            self.sub_(torch.as_tensor(value, dtype=self.dtype).to(self.device))
        _touch(self)
        return self

    def read_value(self):
        return self.detach()

    def value(self):
        return self.detach()

    def numpy(self):
        return self.detach().cpu().numpy()

    def __repr__(self):
        return f"<dtf.Variable '{self.name}' shape={tuple(self.shape)} dtype={self.dtype} device={self.device}>"


def _rebuild_variable(t, trainable, name):
    return Variable(t, trainable=trainable, name=name)


def _touch(v):
    """After a host-side assign, refresh the bf16 shadow if it lives in an arena."""
    s = getattr(v, "_dtf_bf16", None)
    if s is not None and not getattr(v, "_dtf_bf16_owned", False):
        with torch.no_grad():
            s.copy_(v.detach())
    from .ops._util import bump_weights_epoch
    bump_weights_epoch()


ALIGN = 64


def _pad(n):
    return (n + ALIGN - 1) // ALIGN * ALIGN


class ParamArena:
    """Contiguous storage for a list of f32 variables (+ grads, bf16 copies, slots)."""

    def __init__(self, variables, device=None, with_bf16=None, with_grad=True):
        self.variables = list(variables)
        if not self.variables:
            raise ValueError("empty arena")
        self.device = torch.device(device) if device is not None else self.variables[0].device
        self.offsets = []
        off = 0
        for v in self.variables:
            if v.dtype != torch.float32:
                raise TypeError(f"arena variables must be f32 masters ({v.name}: {v.dtype})")
            self.offsets.append(off)
            off += _pad(v.numel())
        self.numel = off
        self.flat = torch.zeros(self.numel, dtype=torch.float32, device=self.device)
        for v, o in zip(self.variables, self.offsets):
            self.flat[o:o + v.numel()].copy_(v.detach().reshape(-1))
            v.data = self.flat[o:o + v.numel()].view(v.shape)
        self.grad = None
        if with_grad:
            self.grad = torch.zeros(self.numel, dtype=torch.float32, device=self.device)
            for v, o in zip(self.variables, self.offsets):
                v.grad = self.grad[o:o + v.numel()].view(v.shape)
                v._dtf_grad_ptr = v.grad.data_ptr()  # ops may accumulate into it directly (ops._util)
        if with_bf16 is None:
            with_bf16 = self.device.type == "cuda"
        self.bf16 = None
        if with_bf16:
            self.bf16 = self.flat.to(torch.bfloat16)
            for v, o in zip(self.variables, self.offsets):
                v._dtf_bf16 = self.bf16[o:o + v.numel()].view(v.shape)
                v._dtf_bf16_owned = False
        self.slots = {}

    def slot(self, name, init=0.0):
        s = self.slots.get(name)
        if s is None:
            s = torch.full((self.numel,), float(init), dtype=torch.float32, device=self.device)
            self.slots[name] = s
        return s

    def slot_view(self, name, var):
        i = self.index(var)
        o = self.offsets[i]
        return self.slots[name][o:o + var.numel()].view(var.shape)

    def index(self, var):
        for i, v in enumerate(self.variables):
            if v is var:
                return i
        raise KeyError(var.name)

    def grad_view(self, i):
        o = self.offsets[i]
        return self.grad[o:o + self.variables[i].numel()]

    def refresh_bf16(self):
        if self.bf16 is not None:
            self.bf16.copy_(self.flat)

    def zero_grad(self):
        if self.grad is not None:
            self.grad.zero_()

    def relink(self):
        """Re-point variables at the arena (after something replaced .data / .grad)."""
        for v, o in zip(self.variables, self.offsets):
            if v.data_ptr() != self.flat[o:].data_ptr():
                self.flat[o:o + v.numel()].copy_(v.detach().reshape(-1))
                v.data = self.flat[o:o + v.numel()].view(v.shape)
            if self.grad is not None:
                v.grad = self.grad[o:o + v.numel()].view(v.shape)
                v._dtf_grad_ptr = v.grad.data_ptr()
