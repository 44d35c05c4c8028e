"""GradientTape: TF-style reverse-mode autodiff over the torch autograd engine.

The reference builds gradients symbolically through ``optimizer.minimize``
(reference trainer/task.py:70,138 -> tf.gradients). Here every op (HIP kernel
or CPU reference) is a torch autograd node with a hand-written backward, and
``GradientTape`` exposes the TF2 surface on top of it.
"""
from __future__ import annotations

import contextlib

import torch


def _flatten(x):
    if isinstance(x, dict):
        return [v for k in sorted(x) for v in _flatten(x[k])]
    if isinstance(x, (list, tuple)):
        return [v for e in x for v in _flatten(e)]
    return [x]


def _unflatten(template, flat):
    it = iter(flat)

    def rec(t):
        if isinstance(t, dict):
            return {k: rec(t[k]) for k in sorted(t)}
        if isinstance(t, (list, tuple)):
            return type(t)(rec(e) for e in t)
        return next(it)
    return rec(template)


class GradientTape(contextlib.AbstractContextManager):
    def __init__(self, persistent=False, watch_accessed_variables=True):
        self.persistent = persistent
        self.watch_accessed_variables = watch_accessed_variables
        self._watched = []
        self._ctx = None
        self._used = False

    def __enter__(self):
        self._ctx = torch.enable_grad()
        self._ctx.__enter__()
        return self

    def __exit__(self, *exc):
        self._ctx.__exit__(*exc)
        return False

    def watch(self, tensor):
        for t in _flatten(tensor):
            if isinstance(t, torch.Tensor) and not t.requires_grad and t.is_floating_point():
                t.requires_grad_(True)
            self._watched.append(t)

    def watched_variables(self):
        return list(self._watched)

    def gradient(self, target, sources, output_gradients=None, unconnected_gradients="none"):
        if self._used and not self.persistent:
            raise RuntimeError("A non-persistent GradientTape can only be used to compute one set of gradients")
        self._used = True
        flat_src = _flatten(sources)
        targets = _flatten(target)
        if output_gradients is not None:
            grads_out = _flatten(output_gradients)
        else:
            grads_out = [torch.ones_like(t) if t.dim() > 0 else None for t in targets]
        need = [s for s in flat_src if isinstance(s, torch.Tensor) and s.requires_grad]
        if need:
            res = torch.autograd.grad([t if t.dim() == 0 or g is not None else t.sum() for t, g in
                                       zip(targets, grads_out)],
                                      need, grad_outputs=[g for g in grads_out], retain_graph=self.persistent,
                                      allow_unused=True)
        else:
            res = []
        it = iter(res)
        out = []
        for s in flat_src:
            g = next(it) if isinstance(s, torch.Tensor) and s.requires_grad else None
            if g is None and unconnected_gradients == "zero":
                g = torch.zeros_like(s)
            out.append(g)
        if isinstance(sources, torch.Tensor):
            return out[0]
        return _unflatten(sources, out)

    def jacobian(self, target, sources):
        return torch.autograd.functional.jacobian(lambda s: target, sources)


def stop_gradient(x):
    return x.detach()
