"""hipGraph capture of training steps (the tf.function / XLA-free answer to per-op launch overhead).

``CapturedStep(fn)`` runs ``fn`` eagerly for ``warmup`` calls, then captures one call into a
hipGraph (``torch.cuda.CUDAGraph`` = hipGraph on ROCm) and afterwards only replays it: every HIP
kernel of forward, backward, (single-rank) gradient reduction and the fused optimizer update is
issued by ONE graph launch. Inputs are copied into static buffers; per-step scalars that the graph
cannot bake in (bias-corrected learning rate, gradient scale) are published by
``Optimizer.graph_prestep`` into the pinned buffers the captured memcpy nodes read; derived weight
layouts are invalidated after every replay. Restrictions (as for any graph capture): static shapes,
no host reads of device values inside the step. Dropout stays random across replays: automatically seeded
dropout kernels also read a device step counter that Model.train_step advances with a captured kernel
(ops._util.advance_rng).
"""
from __future__ import annotations

import torch


def _flat(x, out):
    if isinstance(x, torch.Tensor):
        out.append(x)
    elif isinstance(x, dict):
        for k in sorted(x):
            _flat(x[k], out)
    elif isinstance(x, (list, tuple)):
        for e in x:
            _flat(e, out)
    return out


def _rebuild(template, it):
    if isinstance(template, torch.Tensor):
        return next(it)
    if isinstance(template, dict):
        return {k: _rebuild(template[k], it) for k in sorted(template)}
    if isinstance(template, (list, tuple)):
        return type(template)(_rebuild(e, it) for e in template)
    return template


class CapturedStep:
    def __init__(self, fn, warmup=2, optimizers=(), pool=None):
        self.fn = fn
        self.warmup = warmup
        self.optimizers = list(optimizers)
        self.pool = pool
        self.graph = None
        self.calls = 0
        self.static_in = None
        self.out = None

    def _capture(self, args):
        from .ops import _util
        flat = _flat(args, [])
        self.static_in = [t.clone() for t in flat]
        static_args = _rebuild(args, iter(self.static_in))
        for o in self.optimizers:
            o.graph_prepare()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, pool=self.pool):
            out = self.fn(static_args)
        self.graph = g
        # keep the raw (device) log values: each replay hands out a fresh lazy view of them
        self._log_type = type(out) if isinstance(out, dict) else None
        self.out = {k: dict.__getitem__(out, k) for k in out.keys()} if self._log_type else out
        # the capture did not execute anything: roll the host step back so the first replay is step t
        for o in self.optimizers:
            o._host_iter -= 1
        _util.bump_weights_epoch()

    def __call__(self, args):
        self.calls += 1
        if self.graph is None:
            if self.calls <= self.warmup:
                # warm up on a side stream (lazy inits, allocator pools) as graph capture requires
                cur = torch.cuda.current_stream()
                side = torch.cuda.Stream()
                side.wait_stream(cur)
                with torch.cuda.stream(side):
                    r = self.fn(args)
                cur.wait_stream(side)
                return r
            self._capture(args)
        else:
            for s, t in zip(self.static_in, _flat(args, [])):
                if s.data_ptr() != t.data_ptr():
                    s.copy_(t, non_blocking=True)
        # per-step scalars go to a pinned ring (Optimizer.graph_prestep): no host sync between replays
        for o in self.optimizers:
            o.graph_prestep()
        self.graph.replay()
        for o in self.optimizers:
            o.graph_poststep()
        from .ops import _util
        _util.bump_weights_epoch()
        return self._log_type(self.out) if self._log_type else self.out

    def reset(self):
        for o in self.optimizers:
            o._graph = None
        self.graph = None
        self.calls = 0


def function(fn=None, warmup=2, optimizers=()):
    """Decorator: ``@dtf.function`` captures a (static-shape) step into a hipGraph after `warmup` calls."""
    def wrap(f):
        return CapturedStep(f, warmup=warmup, optimizers=optimizers)
    return wrap(fn) if fn is not None else wrap
