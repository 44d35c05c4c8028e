"""Optimizers with TF1 / Keras semantics on fused multi-tensor HIP kernels.

The reference's optimizer factory (reference trainer/task.py:41-56) maps a
flag string to one of six TF1 optimizers constructed with only a learning
rate; their update rules, defaults and checkpoint slot names are reproduced
here (SURVEY §2.4.a K10–K15):

=========  ==========================================  ===========================
name       TF1 defaults                                slots (checkpoint names)
=========  ==========================================  ===========================
sgd        —                                           — (Momentum: ``Momentum``)
adadelta   rho=0.95, epsilon=1e-8                      ``Adadelta``, ``Adadelta_1``
adagrad    initial_accumulator_value=0.1               ``Adagrad``
adam       beta1=0.9, beta2=0.999, epsilon=1e-8        ``Adam``, ``Adam_1`` + beta powers
ftrl       lr_power=-0.5, init_accum=0.1, l1=l2=0      ``Ftrl``, ``Ftrl_1``
rmsprop    decay=0.9, momentum=0, epsilon=1e-10, ms=1  ``RMSProp``, ``RMSProp_1``
=========  ==========================================  ===========================

On GPU the whole variable set lives in a ``ParamArena`` and every step is ONE
launch of ``dtf_optim_apply`` that also refreshes the bf16 compute copies.
Per-step scalars (bias-corrected lr, gradient scale, clip threshold) go
through a 4-float device buffer so the step stays hipGraph-capturable.
"""
from __future__ import annotations

import math

import numpy as np
import torch

from ..variables import ParamArena, Variable
from ..ops import _util
from ..ops.optim import optim_apply, sumsq as _sumsq

# rows of the pinned per-step scalar ring of a hipGraph-captured step (how far the host may run ahead)
GRAPH_RING = 8

_SLOTS = {
    "sgd": [],
    "momentum": [("Momentum", 0.0)],
    "adam": [("Adam", 0.0), ("Adam_1", 0.0)],
    "adamw": [("Adam", 0.0), ("Adam_1", 0.0)],
    "adagrad": [("Adagrad", None)],
    "adadelta": [("Adadelta", 0.0), ("Adadelta_1", 0.0)],
    "ftrl": [("Ftrl", None), ("Ftrl_1", 0.0)],
    "rmsprop": [("RMSProp", None), ("RMSProp_1", 0.0)],
}
_KERNEL_KIND = {"sgd": 0, "momentum": 0, "adam": 1, "adamw": 1, "adagrad": 2, "adadelta": 3, "ftrl": 4,
                "rmsprop": 5}


class LearningRateSchedule:
    def __call__(self, step):
        raise NotImplementedError


class PolynomialDecay(LearningRateSchedule):
    def __init__(self, initial_learning_rate, decay_steps, end_learning_rate=0.0001, power=1.0, warmup_steps=0):
        self.lr0, self.steps, self.lr1, self.power, self.warm = (initial_learning_rate, decay_steps,
                                                                 end_learning_rate, power, warmup_steps)

    def __call__(self, step):
        if self.warm and step < self.warm:
            return self.lr0 * (step + 1) / self.warm
        s = min(step, self.steps)
        return (self.lr0 - self.lr1) * (1 - s / self.steps) ** self.power + self.lr1


class CosineDecay(LearningRateSchedule):
    def __init__(self, initial_learning_rate, decay_steps, alpha=0.0, warmup_steps=0):
        self.lr0, self.steps, self.alpha, self.warm = initial_learning_rate, decay_steps, alpha, warmup_steps

    def __call__(self, step):
        if self.warm and step < self.warm:
            return self.lr0 * (step + 1) / self.warm
        s = min(step, self.steps)
        c = 0.5 * (1 + math.cos(math.pi * s / self.steps))
        return self.lr0 * ((1 - self.alpha) * c + self.alpha)


class PiecewiseConstantDecay(LearningRateSchedule):
    def __init__(self, boundaries, values):
        self.b, self.v = list(boundaries), list(values)

    def __call__(self, step):
        for b, v in zip(self.b, self.v):
            if step <= b:
                return v
        return self.v[-1]


class Optimizer:
    """Base optimizer: arena-backed fused updates (GPU) / identical torch math (CPU)."""

    kind = "sgd"

    def __init__(self, learning_rate=0.01, name=None, clipnorm=None, global_clipnorm=None, loss_scale=1.0,
                 **hyper):
        self.learning_rate = learning_rate
        self.name = name or type(self).__name__
        self.global_clipnorm = global_clipnorm or clipnorm
        self.loss_scale = float(loss_scale)
        self.hyper = dict(hyper)
        self.iterations = Variable(0, trainable=False, name="iterations", dtype=torch.int64)
        self._arenas = {}      # key: tuple(id(v)) -> ParamArena
        self._hp = {}
        self._grad_scale = 1.0
        self._pinned = None
        self._host_iter = None     # host mirror of `iterations` (no device sync per step)
        self._graph = None         # set while captured in a hipGraph (see graphs.CapturedStep)

    # --------------------------------------------------------------- config
    def _lr_value(self, step=None):
        lr = self.learning_rate
        if isinstance(lr, LearningRateSchedule) or callable(lr):
            return float(lr(self.host_iterations() if step is None else step))
        return float(lr)

    def get_config(self):
        lr = self.learning_rate
        return {"name": self.name, "kind": self.kind, "learning_rate": lr if isinstance(lr, (int, float)) else None,
                **self.hyper}

    def slot_specs(self):
        specs = []
        for nm, init in _SLOTS[self.kind]:
            if init is None:
                init = self.hyper.get("initial_accumulator_value", 0.1) if self.kind in ("adagrad", "ftrl") \
                    else self.hyper.get("ms_init", 1.0)
            specs.append((nm, init))
        return specs

    # --------------------------------------------------------------- arenas
    def arena_for(self, var_list):
        key = tuple(id(v) for v in var_list)
        a = self._arenas.get(key)
        if a is None:
            existing = getattr(var_list[0], "_dtf_arena", None)
            if existing is not None and [id(v) for v in existing.variables] == list(key):
                a = existing
            else:
                a = ParamArena(var_list)
                for v in var_list:
                    v._dtf_arena = a
            for nm, init in self.slot_specs():
                a.slot(nm, init)
            self._arenas[key] = a
        return a

    def build(self, var_list):
        var_list = [v for v in var_list if v.requires_grad]
        if var_list:
            self.arena_for(var_list)
        return self

    def get_slot(self, var, name):
        a = getattr(var, "_dtf_arena", None)
        if a is None:
            raise KeyError(f"{var.name} has no optimizer state")
        return a.slot_view(name, var)

    def get_slot_names(self):
        return [n for n, _ in _SLOTS[self.kind]]

    def variables(self):
        out = [self.iterations]
        for a in self._arenas.values():
            for nm, _ in _SLOTS[self.kind]:
                for v in a.variables:
                    out.append((f"{v.name}/{nm}", a.slot_view(nm, v)))
        return out

    # --------------------------------------------------------------- step math
    def _effective_lr(self, t):
        lr = self._lr_value(t - 1)
        if self.kind in ("adam", "adamw"):
            b1, b2 = self.hyper.get("beta_1", 0.9), self.hyper.get("beta_2", 0.999)
            lr = lr * math.sqrt(1 - b2 ** t) / (1 - b1 ** t)
        return lr

    def _kernel_kwargs(self):
        h = self.hyper
        k = self.kind
        if k in ("sgd", "momentum"):
            return dict(mom=h.get("momentum", 0.0), nesterov=h.get("nesterov", False), wd=h.get("weight_decay", 0.0))
        if k in ("adam", "adamw"):
            return dict(b1=h.get("beta_1", 0.9), b2=h.get("beta_2", 0.999), eps=h.get("epsilon", 1e-8),
                        wd=h.get("weight_decay", 0.0))
        if k == "adagrad":
            return dict(eps=h.get("epsilon", 0.0))
        if k == "adadelta":
            return dict(b1=h.get("rho", 0.95), eps=h.get("epsilon", 1e-8))
        if k == "ftrl":
            return dict(l1=h.get("l1_regularization_strength", 0.0), l2=h.get("l2_regularization_strength", 0.0))
        if k == "rmsprop":
            return dict(b1=h.get("rho", h.get("decay", 0.9)), mom=h.get("momentum", 0.0), eps=h.get("epsilon", 1e-10))
        raise ValueError(k)

    def set_grad_scale(self, s):
        """Scale applied to every gradient inside the fused update (e.g. 1/num_replicas, 1/loss_scale)."""
        self._grad_scale = float(s)

    def host_iterations(self):
        if self._host_iter is None:
            self._host_iter = int(self.iterations.item())
        return self._host_iter

    def reset_host_state(self):
        """After iterations was restored (checkpoint), re-read it."""
        self._host_iter = None

    def _hp_values(self, lr):
        return [lr, self._grad_scale / self.loss_scale, float(self.global_clipnorm or 0.0), 0.0]

    def _hp_tensor(self, a, lr):
        hp = self._hp.get(id(a))
        vals = self._hp_values(lr)
        if self._graph is not None:
            # inside a capture: a pinned ring of GRAPH_RING scalar rows that the host fills before each replay
            # (graph_prestep); the captured copy brings the ring to the device at replay time and a captured
            # select kernel picks row (replay count % GRAPH_RING) with a device counter
            ring = self._graph.get(id(a))
            if ring is None or hp is None:
                raise RuntimeError("optimizer arena was not prepared for graph capture (graph_prepare())")
            pinned, dev_table, ctr = ring
            dev_table.copy_(pinned, non_blocking=True)
            _util.call("dtf_hp_ring_select", _util.ptr(dev_table), GRAPH_RING, 4, _util.ptr(ctr), _util.ptr(hp),
                       _util.stream())
            return hp
        if hp is None:
            hp = torch.tensor(vals, dtype=torch.float32, device=a.device)
            self._hp[id(a)] = hp
            return hp
        if a.device.type == "cuda":
            # ring of pinned staging buffers; a slot is reused only after its copy has executed
            if self._pinned is None:
                self._pinned = [(torch.zeros(4, dtype=torch.float32).pin_memory(), torch.cuda.Event())
                                for _ in range(8)]
                self._ring = 0
            buf, ev = self._pinned[self._ring]
            self._ring = (self._ring + 1) % len(self._pinned)
            ev.synchronize()
            buf.copy_(torch.tensor(vals))
            hp.copy_(buf, non_blocking=True)
            ev.record()
        else:
            hp.copy_(torch.tensor(vals))
        return hp

    def apply_arena(self, a, zero_grad=True):
        """Apply one update to a whole arena whose gradient buffer is already filled."""
        t = self.host_iterations() + 1
        lr = self._effective_lr(t)
        kw = self._kernel_kwargs()
        specs = self.slot_specs()
        s1 = a.slots[specs[0][0]] if len(specs) > 0 else None
        s2 = a.slots[specs[1][0]] if len(specs) > 1 else None
        if a.device.type == "cuda":
            hp = self._hp_tensor(a, lr)
            ss = None
            if self.global_clipnorm:
                ss = torch.empty(1, dtype=torch.float32, device=a.device) if not hasattr(a, "_sumsq") else a._sumsq
                a._sumsq = ss
                _sumsq(a.grad, ss)
            optim_apply(_KERNEL_KIND[self.kind], a.flat, a.grad, s1, s2, a.bf16, hp, zero_grad=zero_grad, sumsq=ss,
                        **kw)
            _util.bump_weights_epoch()
        else:
            gs = self._grad_scale / self.loss_scale
            if self.global_clipnorm:
                n = float(a.grad.norm()) * gs
                if n > self.global_clipnorm:
                    gs *= self.global_clipnorm / n
            _torch_update(_KERNEL_KIND[self.kind], a.flat, a.grad, s1, s2, lr, gs, **kw)
            if zero_grad:
                a.grad.zero_()
        with torch.no_grad():
            self.iterations.add_(1)
        self._host_iter = t

    # ---- bucket-by-bucket update during backward (collective.GradientBucketer with an optimizer attached)
    def supports_ranges(self):
        """Elementwise update rules only: global-norm clipping needs the whole gradient first."""
        return not self.global_clipnorm and self.kind in _KERNEL_KIND

    def begin_step(self, a):
        """Fix this step's scalars (lr, grad scale) before the first range update; the device scalar buffer is
        filled once (in graph mode its ring row is selected once) on the current stream."""
        t = self.host_iterations() + 1
        lr = self._effective_lr(t)
        hp = self._hp_tensor(a, lr) if a.device.type == "cuda" else None
        self._range_step = (t, lr, hp)

    def apply_range(self, a, lo, hi):
        """Update arena elements [lo, hi) (whole variables) and zero their gradients."""
        t, lr, hp = self._range_step
        kw = self._kernel_kwargs()
        specs = self.slot_specs()
        s1 = a.slots[specs[0][0]][lo:hi] if len(specs) > 0 else None
        s2 = a.slots[specs[1][0]][lo:hi] if len(specs) > 1 else None
        if a.device.type == "cuda":
            optim_apply(_KERNEL_KIND[self.kind], a.flat[lo:hi], a.grad[lo:hi], s1, s2,
                        None if a.bf16 is None else a.bf16[lo:hi], hp, zero_grad=True, **kw)
        else:
            _torch_update(_KERNEL_KIND[self.kind], a.flat[lo:hi], a.grad[lo:hi], s1, s2, lr,
                          self._grad_scale / self.loss_scale, **kw)
            a.grad[lo:hi].zero_()

    def end_step(self, a):
        t = self._range_step[0]
        self._range_step = None
        if a.device.type == "cuda":
            _util.bump_weights_epoch()
        with torch.no_grad():
            self.iterations.add_(1)
        self._host_iter = t

    def apply_segments(self, a, segments, reduce_sumsq=None):
        """One update of the arena ranges this replica owns (ZeRO-1, parallel.collective.ShardedGradientBucketer):
        ``segments`` = [(lo, hi, grad)] with ``grad`` the summed gradient of arena elements [lo, hi); masters,
        slots and bf16 copies are updated in place over those ranges only, one fused launch per segment.
        ``reduce_sumsq(t)`` sums a 1-element tensor over the replicas (global-norm clipping needs the norm of
        the WHOLE gradient, of which each replica holds a part)."""
        if self.kind == "lamb":
            raise ValueError("LAMB's per-variable trust ratio cannot be applied to sharded optimizer state")
        t = self.host_iterations() + 1
        lr = self._effective_lr(t)
        kw = self._kernel_kwargs()
        specs = self.slot_specs()
        s1 = a.slots[specs[0][0]] if len(specs) > 0 else None
        s2 = a.slots[specs[1][0]] if len(specs) > 1 else None
        sl = lambda s, lo, hi: None if s is None else s[lo:hi]  # noqa: E731
        if a.device.type == "cuda":
            hp = self._hp_tensor(a, lr)
            ss = None
            if self.global_clipnorm:
                ss = getattr(a, "_sumsq", None)
                if ss is None:
                    ss = a._sumsq = torch.empty(1, dtype=torch.float32, device=a.device)
                ss.zero_()
                for _, _, g in segments:
                    _sumsq(g, ss, zero=False)
                if reduce_sumsq is not None:
                    reduce_sumsq(ss)
            for lo, hi, g in segments:
                optim_apply(_KERNEL_KIND[self.kind], a.flat[lo:hi], g, sl(s1, lo, hi), sl(s2, lo, hi),
                            sl(a.bf16, lo, hi), hp, zero_grad=True, sumsq=ss, **kw)
            _util.bump_weights_epoch()
        else:
            gs = self._grad_scale / self.loss_scale
            if self.global_clipnorm:
                n2 = torch.zeros(1, dtype=torch.float64)
                for _, _, g in segments:
                    n2 += (g.double() ** 2).sum()
                if reduce_sumsq is not None:
                    reduce_sumsq(n2)
                n = float(n2.sqrt()) * gs
                if n > self.global_clipnorm:
                    gs *= self.global_clipnorm / n
            for lo, hi, g in segments:
                _torch_update(_KERNEL_KIND[self.kind], a.flat[lo:hi], g, sl(s1, lo, hi), sl(s2, lo, hi), lr, gs, **kw)
                g.zero_()
        with torch.no_grad():
            self.iterations.add_(1)
        self._host_iter = t

    def graph_prepare(self):
        """Allocate (outside the capture: pinned allocation is not capturable) the fixed pinned
        scalar buffer and device hp tensor of every arena, and switch `_hp_tensor` to graph mode."""
        self._graph = {}
        self._graph_replays = 0
        self._graph_events = [None] * GRAPH_RING
        for a in self._arenas.values():
            if a.device.type != "cuda":
                continue
            self._graph[id(a)] = (torch.zeros(GRAPH_RING, 4, dtype=torch.float32).pin_memory(),
                                  torch.zeros(GRAPH_RING, 4, dtype=torch.float32, device=a.device),
                                  torch.zeros(1, dtype=torch.int32, device=a.device))
            if id(a) not in self._hp:
                self._hp[id(a)] = torch.zeros(4, dtype=torch.float32, device=a.device)

    def graph_prestep(self):
        """Before a hipGraph replay of a captured step: advance the host step and publish the step's
        scalars (bias-corrected lr, grad scale, clip) into this replay's row of the pinned ring. The host
        blocks only when it is GRAPH_RING replays ahead of the GPU (the row's previous reader not done)."""
        t = self.host_iterations() + 1
        lr = self._effective_lr(t)
        slot = self._graph_replays % GRAPH_RING
        ev = self._graph_events[slot]
        if ev is not None:
            ev.synchronize()
        vals = torch.tensor(self._hp_values(lr))
        for pinned, _, _ in (self._graph or {}).values():
            pinned[slot].copy_(vals)
        self._host_iter = t
        if not self.iterations.is_cuda:  # host-resident counter: the capture ran its add_ only once
            with torch.no_grad():
                self.iterations.fill_(t)

    def graph_poststep(self):
        """After a replay was issued: mark its ring row busy until the replay has run."""
        if self._graph is None:
            return
        slot = self._graph_replays % GRAPH_RING
        ev = self._graph_events[slot]
        if ev is None:
            ev = self._graph_events[slot] = torch.cuda.Event()
        ev.record()
        self._graph_replays += 1

    def apply_gradients(self, grads_and_vars, zero_grad=True):
        gv = [(g, v) for g, v in grads_and_vars if g is not None]
        if not gv:
            return
        var_list = [v for _, v in gv]
        a = self.arena_for(var_list)
        for i, (g, v) in enumerate(gv):
            dst = a.grad_view(i).view(v.shape)
            if g.data_ptr() != dst.data_ptr():
                dst.copy_(g.detach().to(torch.float32))
        self.apply_arena(a, zero_grad=zero_grad)

    def minimize(self, loss, var_list, tape=None):
        if callable(loss) and tape is None:
            from ..autodiff import GradientTape
            with GradientTape() as tape:
                value = loss()
            loss = value
        if tape is not None:
            grads = tape.gradient(loss, var_list)
        else:
            grads = torch.autograd.grad(loss, var_list, allow_unused=True)
        self.apply_gradients(zip(grads, var_list))
        return loss


def _torch_update(kind, p, g, s1, s2, lr, gs, b1=0.9, b2=0.999, eps=1e-8, wd=0.0, mom=0.0, l1=0.0, l2=0.0,
                  nesterov=False):
    """Exact torch mirror of the HIP kernel (CPU arenas)."""
    with torch.no_grad():
        g = g * gs
        if kind == 0:
            if wd:
                g = g + wd * p
            if mom:
                s1.mul_(mom).add_(g)
                p.sub_(lr * (g + mom * s1 if nesterov else s1))
            else:
                p.sub_(lr * g)
        elif kind == 1:
            s1.mul_(b1).add_((1 - b1) * g)
            s2.mul_(b2).add_((1 - b2) * g * g)
            p.sub_(lr * (s1 / (s2.sqrt() + eps) + wd * p))
        elif kind == 2:
            s1.add_(g * g)
            p.sub_(lr * g / (s1.sqrt() + eps))
        elif kind == 3:
            s1.mul_(b1).add_((1 - b1) * g * g)
            d = (s2 + eps).sqrt() / (s1 + eps).sqrt() * g
            s2.mul_(b1).add_((1 - b1) * d * d)
            p.sub_(lr * d)
        elif kind == 4:
            n_new = s1 + g * g
            sigma = (n_new.sqrt() - s1.sqrt()) / lr
            s2.add_(g - sigma * p)
            s1.copy_(n_new)
            quad = n_new.sqrt() / lr + 2 * l2
            p.copy_(torch.where(s2.abs() > l1, (torch.sign(s2) * l1 - s2) / quad, torch.zeros_like(p)))
        elif kind == 5:
            s1.mul_(b1).add_((1 - b1) * g * g)
            s2.mul_(mom).add_(lr * g / (s1 + eps).sqrt())
            p.sub_(s2)


# ----------------------------------------------------------------- concrete classes
class SGD(Optimizer):
    kind = "sgd"

    def __init__(self, learning_rate=0.01, momentum=0.0, nesterov=False, weight_decay=0.0, **kw):
        super().__init__(learning_rate, momentum=momentum, nesterov=nesterov, weight_decay=weight_decay, **kw)
        if momentum:
            self.kind = "momentum"


class Adam(Optimizer):
    kind = "adam"

    def __init__(self, learning_rate=0.001, beta_1=0.9, beta_2=0.999, epsilon=1e-7, **kw):
        super().__init__(learning_rate, beta_1=beta_1, beta_2=beta_2, epsilon=epsilon, **kw)


class AdamW(Optimizer):
    kind = "adamw"

    def __init__(self, learning_rate=0.001, weight_decay=0.004, beta_1=0.9, beta_2=0.999, epsilon=1e-7, **kw):
        super().__init__(learning_rate, beta_1=beta_1, beta_2=beta_2, epsilon=epsilon, weight_decay=weight_decay, **kw)


class Adagrad(Optimizer):
    kind = "adagrad"

    def __init__(self, learning_rate=0.001, initial_accumulator_value=0.1, epsilon=1e-7, **kw):
        super().__init__(learning_rate, initial_accumulator_value=initial_accumulator_value, epsilon=epsilon, **kw)


class Adadelta(Optimizer):
    kind = "adadelta"

    def __init__(self, learning_rate=0.001, rho=0.95, epsilon=1e-7, **kw):
        super().__init__(learning_rate, rho=rho, epsilon=epsilon, **kw)


class Ftrl(Optimizer):
    kind = "ftrl"

    def __init__(self, learning_rate=0.001, learning_rate_power=-0.5, initial_accumulator_value=0.1,
                 l1_regularization_strength=0.0, l2_regularization_strength=0.0, **kw):
        if learning_rate_power != -0.5:
            raise NotImplementedError("only learning_rate_power=-0.5 (TF1 default) is fused")
        super().__init__(learning_rate, initial_accumulator_value=initial_accumulator_value,
                         l1_regularization_strength=l1_regularization_strength,
                         l2_regularization_strength=l2_regularization_strength, **kw)


class RMSprop(Optimizer):
    kind = "rmsprop"

    def __init__(self, learning_rate=0.001, rho=0.9, momentum=0.0, epsilon=1e-10, ms_init=1.0, **kw):
        super().__init__(learning_rate, rho=rho, momentum=momentum, epsilon=epsilon, ms_init=ms_init, **kw)


# TF1 constructors with TF1 defaults (reference trainer/task.py:42-53)
def GradientDescentOptimizer(learning_rate, **kw):
    return SGD(learning_rate, name="GradientDescent", **kw)


def AdadeltaOptimizer(learning_rate=0.001, rho=0.95, epsilon=1e-8, **kw):
    return Adadelta(learning_rate, rho=rho, epsilon=epsilon, name="Adadelta", **kw)


def AdagradOptimizer(learning_rate, initial_accumulator_value=0.1, **kw):
    return Adagrad(learning_rate, initial_accumulator_value=initial_accumulator_value, epsilon=0.0, name="Adagrad",
                   **kw)


def AdamOptimizer(learning_rate=0.001, beta1=0.9, beta2=0.999, epsilon=1e-8, **kw):
    return Adam(learning_rate, beta_1=beta1, beta_2=beta2, epsilon=epsilon, name="Adam", **kw)


def FtrlOptimizer(learning_rate, learning_rate_power=-0.5, initial_accumulator_value=0.1,
                  l1_regularization_strength=0.0, l2_regularization_strength=0.0, **kw):
    return Ftrl(learning_rate, learning_rate_power, initial_accumulator_value, l1_regularization_strength,
                l2_regularization_strength, name="Ftrl", **kw)


def RMSPropOptimizer(learning_rate, decay=0.9, momentum=0.0, epsilon=1e-10, **kw):
    return RMSprop(learning_rate, rho=decay, momentum=momentum, epsilon=epsilon, ms_init=1.0, name="RMSProp", **kw)


def MomentumOptimizer(learning_rate, momentum, use_nesterov=False, **kw):
    return SGD(learning_rate, momentum=momentum, nesterov=use_nesterov, name="Momentum", **kw)


_TF1_FACTORY = {
    "sgd": GradientDescentOptimizer,
    "adadelta": AdadeltaOptimizer,
    "adagrad": AdagradOptimizer,
    "adam": AdamOptimizer,
    "ftrl": FtrlOptimizer,
    "rmsprop": RMSPropOptimizer,
}

_KERAS = {"sgd": SGD, "adam": Adam, "adamw": AdamW, "adagrad": Adagrad, "adadelta": Adadelta, "ftrl": Ftrl,
          "rmsprop": RMSprop}


def get(identifier, learning_rate=None, tf1=True, **kw):
    """String -> optimizer. tf1=True reproduces reference trainer/task.py:41-56 (TF1 defaults)."""
    if isinstance(identifier, Optimizer):
        return identifier
    name = str(identifier).lower()
    if tf1 and name in _TF1_FACTORY:
        return _TF1_FACTORY[name](0.01 if learning_rate is None else learning_rate, **kw)
    if name in _KERAS:
        cls = _KERAS[name]
        return cls(**({} if learning_rate is None else {"learning_rate": learning_rate}), **kw)
    raise ValueError(f"Unknown optimizer: {identifier}")


# ----------------------------------------------------------------- test oracles
def reference_update(kind, p, grads, lr=0.01):
    """Sequential numpy oracle of the TF1 update rules with TF1 defaults."""
    p = p.double().numpy().copy()
    z = np.zeros_like(p)
    s1, s2 = z.copy(), z.copy()
    if kind in ("adagrad", "ftrl"):
        s1[:] = 0.1
    if kind == "rmsprop":
        s1[:] = 1.0
    for t, g in enumerate(grads, 1):
        g = g.double().numpy()
        if kind == "sgd":
            p -= lr * g
        elif kind == "adam":
            s1 = 0.9 * s1 + 0.1 * g
            s2 = 0.999 * s2 + 0.001 * g * g
            lrt = lr * math.sqrt(1 - 0.999 ** t) / (1 - 0.9 ** t)
            p -= lrt * s1 / (np.sqrt(s2) + 1e-8)
        elif kind == "adagrad":
            s1 += g * g
            p -= lr * g / np.sqrt(s1)
        elif kind == "adadelta":
            s1 = 0.95 * s1 + 0.05 * g * g
            d = np.sqrt(s2 + 1e-8) / np.sqrt(s1 + 1e-8) * g
            s2 = 0.95 * s2 + 0.05 * d * d
            p -= lr * d
        elif kind == "ftrl":
            n_new = s1 + g * g
            sigma = (np.sqrt(n_new) - np.sqrt(s1)) / lr
            s2 += g - sigma * p
            s1 = n_new
            quad = np.sqrt(n_new) / lr
            p = np.where(np.abs(s2) > 0, -s2 / quad, 0.0)
        elif kind == "rmsprop":
            s1 = 0.9 * s1 + 0.1 * g * g
            s2 = 0.0 * s2 + lr * g / np.sqrt(s1 + 1e-10)
            p -= s2
    return torch.from_numpy(p).float()


def fused_update_for_test(opt, p, grads):
    v = Variable(p.clone(), name="w")
    for g in grads:
        opt.apply_gradients([(g, v)])
    return v.detach()
