"""Keras Model / Sequential with compile / fit / evaluate / predict.

The training step (``train_step``) is the MI355X hot path:
  forward (bf16 HIP kernels) -> loss -> backward, whose gradients accumulate
  straight into the model's flat f32 gradient arena while the strategy's
  bucketed RCCL all-reduce runs behind it -> ONE fused optimizer launch that
  also refreshes the bf16 weight copies and zeroes the gradients.
No host synchronisation happens inside a step: losses and metrics stay on the
device until an epoch ends or a callback asks for a value.

Reference parity: the reference's per-epoch evaluation on sample 0 and
``Epoch: i, loss: ...`` print every ``checkpoint_period`` epochs
(reference trainer/task.py:89-96) is provided by the training CLI
(cli/train.py) on top of this loop.
"""
from __future__ import annotations

import copy
import math
import os
import time

import numpy as np
import torch

from .. import context
from .. import profiler as prof
from ..ops._util import advance_rng, direct_grads, join_side_streams
from ..data import Dataset
from ..parallel import strategy as S
from . import callbacks as cbs
from . import losses as L
from . import metrics as M
from . import optimizers as O
from . import layers as KL
from .layers import InputLayer, Layer


class _LazyLogs(dict):
    """Logs whose tensor values are converted to floats only when read."""

    def __getitem__(self, k):
        v = dict.__getitem__(self, k)
        if isinstance(v, torch.Tensor):
            v = float(v.detach().float().item())
            dict.__setitem__(self, k, v)
        return v

    def get(self, k, d=None):
        return self[k] if k in self else d

    def items(self):
        return [(k, self[k]) for k in self.keys()]

    def values(self):
        return [self[k] for k in self.keys()]

    def materialize(self):
        return {k: self[k] for k in self.keys()}


def _to_device_tensor(x, dev):
    if x is None:
        return None
    if isinstance(x, dict):
        return {k: _to_device_tensor(v, dev) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return type(x)(_to_device_tensor(v, dev) for v in x)
    t = x if isinstance(x, torch.Tensor) else torch.as_tensor(np.asarray(x))
    if t.dtype == torch.float64:
        t = t.float()
    return t.to(dev, non_blocking=True)


def _unpack(data):
    if isinstance(data, (tuple, list)):
        if len(data) == 1:
            return data[0], None, None
        if len(data) == 2:
            return data[0], data[1], None
        return data[0], data[1], data[2]
    return data, None, None


def _head(x, n=1):
    """The first n samples of a (possibly nested) input batch: enough to build lazily created weights."""
    if isinstance(x, torch.Tensor):
        return x[:n]
    if isinstance(x, dict):
        return {k: _head(v, n) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return type(x)(_head(v, n) for v in x)
    return x


class Model(Layer):
    # run the optimizer bucket by bucket during backward (parallel.strategy._OVERLAP_UPDATE); models whose
    # backward leaves CUs idle opt in
    overlap_update = False

    def __init__(self, inputs=None, outputs=None, name=None, **kw):
        super().__init__(name=name, **kw)
        self.optimizer = None
        self.compiled_loss = None
        self.compiled_metrics = []
        self.stop_training = False
        self._arena = None
        self._strategy = None
        self._is_chief = True
        self._initial_epoch = 0
        self.history = None
        self._replicas = {}
        self._graph = None
        if inputs is not None or outputs is not None:
            self._init_graph(inputs, outputs)

    # ------------------------------------------------------------ functional graph
    def _init_graph(self, inputs, outputs):
        """Model(inputs=..., outputs=...): inputs/outputs are KerasTensors (keras.Input and layer outputs), single
        or nested in lists/tuples/dicts. The nodes between them are kept in topological order; call() evaluates
        them, so training, saving and the strategies treat the graph like any other model."""
        if inputs is None or outputs is None:
            raise ValueError("a functional Model needs both inputs and outputs")
        ins = KL._flatten(inputs)
        if not all(isinstance(t, KL.KerasTensor) and t.layer is None for t in ins):
            raise ValueError("Model inputs must be keras.Input tensors")
        order, seen, layers = [], set(), []

        def visit(t):
            if not isinstance(t, KL.KerasTensor) or id(t) in seen:
                return
            seen.add(id(t))
            if t.layer is None:
                if all(t is not i for i in ins):
                    raise ValueError(f"{t} is not reachable from the model inputs")
                return
            for u in KL._flatten(t.inputs):
                visit(u)
            order.append(t)
            if t.layer not in layers:
                layers.append(t.layer)

        for t in KL._flatten(outputs):
            if not isinstance(t, KL.KerasTensor):
                raise ValueError("Model outputs must be KerasTensors")
            visit(t)
        self._graph = (inputs, outputs, order)
        for l in layers:
            if l not in self._layers:
                self._layers.append(l)
        self.built = True

    def _run_graph(self, x, training):
        inputs, outputs, order = self._graph
        env = {}
        if isinstance(inputs, KL.KerasTensor):
            env[id(inputs)] = x
        elif isinstance(inputs, dict):
            if not isinstance(x, dict):
                raise ValueError(f"this model takes a dict of inputs {sorted(inputs)}")
            for k, t in inputs.items():
                env[id(t)] = x[k]
        else:
            xs = KL._flatten(x) if not isinstance(x, torch.Tensor) else [x]
            flat = KL._flatten(inputs)
            if len(xs) != len(flat):
                raise ValueError(f"expected {len(flat)} inputs, got {len(xs)}")
            for t, v in zip(flat, xs):
                env[id(t)] = v
        done = {}  # one evaluation per node: the outputs of a multi-output layer share their node
        for t in order:
            nd = t.node
            if id(nd) not in done:
                args = KL._map_structure(lambda u: env[id(u)] if isinstance(u, KL.KerasTensor) else u, nd.inputs)
                kw = dict(nd.kwargs)
                if KL._takes_training(nd.layer):
                    kw["training"] = training
                done[id(nd)] = nd.layer(args, *nd.args, **kw)
            out = done[id(nd)]
            for p in (t.index or ()):
                out = out[p]
            env[id(t)] = out
        return KL._map_structure(lambda t: env[id(t)], outputs)

    def get_layer(self, name=None, index=None):
        """A direct sublayer by name or position (Keras Model.get_layer)."""
        if index is not None:
            return self.layers[index]
        for l in self.layers:
            if l.name == name:
                return l
        raise ValueError(f"no layer named {name!r} in {self.name}")

    def call(self, inputs, training=None):
        if self._graph is None:
            raise NotImplementedError("subclassed models implement call(); functional models pass inputs/outputs")
        return self._run_graph(inputs, training)

    # ------------------------------------------------------------ compile
    def compile(self, optimizer="rmsprop", loss=None, metrics=None, loss_weights=None, steps_per_execution=1,
                jit_compile=False, **kw):
        self.optimizer = O.get(optimizer, tf1=False) if isinstance(optimizer, str) else optimizer
        self.compiled_loss = L.get(loss)
        self.compiled_metrics = [M.get(m) for m in (metrics or [])]
        self._loss_tracker = M.Mean("loss")
        self._strategy = S.get_strategy()
        self._is_chief = self._strategy.is_chief
        self._jit = bool(jit_compile)
        self._train_fn = None

    @property
    def distribute_strategy(self):
        return self._strategy or S.get_strategy()

    @property
    def metrics(self):
        return [self._loss_tracker] + self.compiled_metrics

    @property
    def metrics_names(self):
        return [m.name for m in self.metrics]

    # ------------------------------------------------------------ arena / strategy
    def _ensure_arena(self):
        if self._arena is None:
            tv = self.distribute_strategy.order_variables(self.trainable_variables)
            if not tv:
                return None
            self.optimizer.build(tv)
            self._arena = self.optimizer.arena_for(tv)
            self.distribute_strategy.setup_model(self, self._arena)
        return self._arena

    def _fully_built(self):
        def rec(layer):
            return layer.built and all(rec(c) for c in layer._layers)
        return rec(self)

    def compute_loss(self, x=None, y=None, y_pred=None, sample_weight=None):
        loss = self.compiled_loss(y, y_pred, sample_weight) if self.compiled_loss is not None else y_pred.sum()
        reg = getattr(self, "losses", None)
        if reg:
            loss = loss + sum(reg)
        return loss

    def _device(self):
        return self.distribute_strategy.device

    # ------------------------------------------------------------ steps
    def train_step(self, data):
        x, y, sw = _unpack(data)
        strat = self.distribute_strategy
        reps = strat.inproc_replicas() if hasattr(strat, "inproc_replicas") else None
        if reps:
            return self._train_step_inproc(x, y, sw, reps)
        if self._arena is None:
            # lay out the arena (and let the strategy broadcast rank 0's initial state) BEFORE the first
            # forward: otherwise every replica's first gradients come from its own, unsynchronised weights
            if not self._fully_built():
                with torch.no_grad():
                    self(_head(x), training=False)
            self._ensure_arena()
        dev = self._device()
        if dev.type == "cuda":
            advance_rng(dev)  # fresh dropout masks for this step, also under hipGraph replay
        with prof.phase("forward"):
            y_pred = self(x, training=True)
            loss = self.compute_loss(x, y, y_pred, sw)
        arena = self._ensure_arena()
        with prof.phase("backward"), direct_grads():  # includes the overlapped bucket all-reduces
            # per-bucket update during backward when the model asks for it (overlap_update) or DTF_OVERLAP_UPDATE
            # forces it; a step captured as ONE multi-branch hipGraph (and its eager warmups) keeps the single update
            # after backward, the per-stream capture (graphs.SPLIT_DEFAULT) keeps the per-bucket one
            from ..parallel import strategy as _S
            from .. import graphs as _G
            ovl = _S._OVERLAP_UPDATE in ("1", "force") or (_S._OVERLAP_UPDATE == "" and self.overlap_update)
            graph_ok = not getattr(self, "_graph_step", False) or _G.SPLIT_DEFAULT
            strat.backward(loss, arena, optimizer=self.optimizer if ovl and graph_ok else None)
            join_side_streams()  # weight gradients issued on the side stream are in the arena
        with prof.phase("optimizer"):
            strat.apply_gradients(self.optimizer, arena)
        return self._update_metrics(loss, y, y_pred)

    def make_train_function(self, force=False):
        """The per-batch step fit() drives. With ``compile(jit_compile=True)`` on a GPU it is a hipGraph-captured
        step (graphs.CapturedStep): eager warmup, one capture, then one graph launch per stream per step. A
        multi-rank step is captured too when its gradient collectives run on the framework's RCCL communicator
        (the per-stream capture puts them in the communication stream's graph); with torch.distributed
        process-group collectives (CommunicationImplementation.RING, ZeRO-1) it stays eager. DTF_GRAPH_DIST=0
        keeps every multi-rank step eager. In-process replicas are never captured."""
        if getattr(self, "_train_fn", None) is not None and not force:
            return self._train_fn
        strat = self.distribute_strategy
        fn = self.train_step
        dev = self._device()
        inproc = bool(strat.inproc_replicas() if hasattr(strat, "inproc_replicas") else None)
        multi = getattr(strat, "_world", 1) > 1 or bool(getattr(strat, "_force", False))
        if getattr(self, "_jit", False) and dev.type == "cuda" and not inproc and (
                not multi or os.environ.get("DTF_GRAPH_DIST", "1") != "0"):
            from ..graphs import CapturedStep
            fn = CapturedStep(self.train_step, warmup=2, optimizers=[self.optimizer], require_split=multi)
        self._graph_step = type(fn).__name__ == "CapturedStep"
        self._train_fn = fn
        return fn

    def _update_metrics(self, loss, y, y_pred):
        with torch.no_grad():
            self._loss_tracker.update_state(loss.detach())
            for m in self.compiled_metrics:
                if y is not None:
                    m.update_state(y, y_pred.detach())
        logs = _LazyLogs(loss=loss.detach())
        return logs

    def _train_step_inproc(self, x, y, sw, devices):
        """In-process MirroredStrategy over several local devices."""
        if self._arena is None and not self.built:
            with torch.no_grad():  # build the variables before the arena is laid out
                self(x[:1].to(devices[0]), training=False)
        arena = self._ensure_arena()
        R = len(devices)
        n = x.shape[0]
        per = n // R
        total = 0.0
        preds = []
        primary = devices[0]
        for r, d in enumerate(devices):
            xs = x[r * per:(r + 1) * per]
            ys = y[r * per:(r + 1) * per] if y is not None else None
            rep = self._replica_for(d, primary)
            xs = xs.to(d)
            ys = ys.to(d) if ys is not None else None
            yp = rep(xs, training=True)
            loss = self.compute_loss(xs, ys, yp, None)
            loss.backward()
            if rep is not self:
                # ReductionToOneDevice: add the replica's gradients into the primary arena
                for v, rv in zip(self.trainable_variables, rep.trainable_variables):
                    if rv.grad is not None:
                        v.grad.add_(rv.grad.to(v.device))
                        rv.grad = None
            total = total + loss.detach().to(primary)
            preds.append(yp.detach().to(primary))
        self.optimizer.set_grad_scale(1.0 / R)
        self.optimizer.apply_arena(arena, zero_grad=True)
        for d, rep in self._replicas.items():
            if rep is not self:
                with torch.no_grad():
                    for v, rv in zip(self.variables, rep.variables):
                        rv.copy_(v.to(rv.device))
        loss = total / R
        return self._update_metrics(loss, y.to(primary) if y is not None else None, torch.cat(preds))

    def _replica_for(self, dev, primary):
        if dev == primary or (dev.type == "cpu" and primary.type == "cpu"):
            return self
        rep = self._replicas.get(dev)
        if rep is None:
            rep = copy.deepcopy(self)
            rep._replicas = {}
            with torch.no_grad():
                for v in rep.variables:
                    v.data = v.data.to(dev)
            self._replicas[dev] = rep
        return rep

    def test_step(self, data):
        x, y, sw = _unpack(data)
        with torch.no_grad():
            y_pred = self(x, training=False)
            loss = self.compute_loss(x, y, y_pred, sw)
            return self._update_metrics(loss, y, y_pred)

    def predict_step(self, data):
        x, _, _ = _unpack(data)
        with torch.no_grad():
            return self(x, training=False)

    # ------------------------------------------------------------ data plumbing
    def _make_dataset(self, x, y, sample_weight, batch_size, shuffle, seed=0):
        strat = self.distribute_strategy
        if isinstance(x, Dataset):
            ds = strat.experimental_distribute_dataset(x) if getattr(strat, "_world", 1) > 1 else x
            return ds, None
        n = (x[0] if isinstance(x, (list, tuple)) else x).shape[0]
        bs = batch_size or 32
        sl_world = getattr(strat, "_world", 1)
        rank = getattr(strat, "_rank", 0)

        def gen(epoch):
            idx = np.arange(n)
            if shuffle:
                np.random.default_rng(seed + epoch).shuffle(idx)
            for s in range(0, n, bs):
                b = idx[s:s + bs]
                if sl_world > 1:  # global batch split across replicas
                    per = len(b) // sl_world
                    if per == 0:
                        continue
                    b = b[rank * per:(rank + 1) * per]
                b = torch.as_tensor(b)
                xb = x[b] if not isinstance(x, (list, tuple)) else type(x)(t[b] for t in x)
                yb = y[b] if y is not None else None
                swb = sample_weight[b] if sample_weight is not None else None
                yield (xb, yb) if swb is None else (xb, yb, swb)
        steps = math.ceil(n / bs)
        return gen, steps

    def _prep_xy(self, x, y, sample_weight):
        def tt(a):
            if a is None or isinstance(a, Dataset):
                return a
            if isinstance(a, (list, tuple)) and a and not np.isscalar(a[0]):
                return type(a)(tt(e) for e in a)
            t = a if isinstance(a, torch.Tensor) else torch.as_tensor(np.asarray(a))
            return t.float() if t.dtype == torch.float64 else t
        return tt(x), tt(y), tt(sample_weight)

    # ------------------------------------------------------------ fit / evaluate / predict
    def fit(self, x=None, y=None, batch_size=None, epochs=1, verbose=1, callbacks=None, validation_split=0.0,
            validation_data=None, shuffle=True, initial_epoch=0, steps_per_epoch=None, validation_steps=None,
            sample_weight=None, validation_freq=1, **kw):
        if self.optimizer is None:
            raise RuntimeError("compile() the model before fit()")
        x, y, sample_weight = self._prep_xy(x, y, sample_weight)
        if validation_split and not isinstance(x, Dataset):
            n = x.shape[0]
            k = int(n * (1 - validation_split))
            validation_data = (x[k:], y[k:])
            x, y = x[:k], y[:k]
        dev = self._device()
        self.history = cbs.History()
        cb_list = list(callbacks or [])
        if verbose:
            cb_list.append(cbs.ProgbarLogger(verbose))
        cb_list.append(self.history)
        cbl = cbs.CallbackList(cb_list, model=self, params={"epochs": epochs, "verbose": verbose})
        self.stop_training = False
        self._initial_epoch = initial_epoch
        cbl.on_train_begin()
        start_epoch = max(initial_epoch, self._initial_epoch)
        src, steps = self._make_dataset(x, y, sample_weight, batch_size, shuffle)
        if steps_per_epoch is not None:
            steps = steps_per_epoch
        ds_iter = None
        train_fn = self.make_train_function()
        for epoch in range(start_epoch, epochs):
            for m in self.metrics:
                m.reset_state()
            cbl.on_epoch_begin(epoch)
            it = src(epoch) if callable(src) else None
            if it is None:
                if ds_iter is None or steps_per_epoch is None:
                    ds_iter = iter(src)
                it = ds_iter
            step = 0
            for data in it:
                cbl.on_train_batch_begin(step)
                data = _to_device_tensor(data, dev)
                logs = train_fn(data)
                cbl.on_train_batch_end(step, logs)
                step += 1
                if self.stop_training or (steps is not None and step >= steps):
                    break
            epoch_logs = self._epoch_logs()
            if validation_data is not None and (epoch + 1) % validation_freq == 0:
                vx, vy = validation_data[0], validation_data[1] if len(validation_data) > 1 else None
                val = self.evaluate(vx, vy, batch_size=batch_size, verbose=0, return_dict=True,
                                    steps=validation_steps)
                epoch_logs.update({f"val_{k}": v for k, v in val.items()})
            cbl.on_epoch_end(epoch, epoch_logs)
            if self.stop_training:
                break
        cbl.on_train_end()
        return self.history

    def _epoch_logs(self):
        out = {}
        strat = self.distribute_strategy
        for m in self.metrics:
            v = m.result()
            if getattr(strat, "_world", 1) > 1:
                v = float(strat.reduce("mean", torch.tensor(v, device=self._device())))
            out[m.name] = v
        return out

    def evaluate(self, x=None, y=None, batch_size=None, verbose=1, sample_weight=None, steps=None, callbacks=None,
                 return_dict=False, **kw):
        x, y, sample_weight = self._prep_xy(x, y, sample_weight)
        dev = self._device()
        for m in self.metrics if self.compiled_loss is not None else []:
            m.reset_state()
        src, nsteps = self._make_dataset(x, y, sample_weight, batch_size, False)
        it = src(0) if callable(src) else iter(src)
        for i, data in enumerate(it):
            if steps is not None and i >= steps:
                break
            self.test_step(_to_device_tensor(data, dev))
        out = self._epoch_logs()
        if verbose:
            print(" - ".join(f"{k}: {v:.4f}" for k, v in out.items()))
        if return_dict:
            return out
        vals = list(out.values())
        return vals[0] if len(vals) == 1 else vals

    def predict(self, x, batch_size=None, verbose=0, steps=None, **kw):
        x, _, _ = self._prep_xy(x, None, None)
        dev = self._device()
        outs = []
        if isinstance(x, Dataset):
            it = iter(x)
        else:
            n = x.shape[0]
            bs = batch_size or 32
            it = ((x[s:s + bs],) for s in range(0, n, bs))
        for i, data in enumerate(it):
            if steps is not None and i >= steps:
                break
            outs.append(self.predict_step(_to_device_tensor(data, dev)).float().cpu())
        return torch.cat(outs).numpy() if outs else np.zeros((0,))

    def __call__(self, inputs, *args, **kwargs):
        if self._graph is not None:  # functional: lists / dicts are the model's input structure
            inputs = KL._map_structure(lambda v: torch.as_tensor(v) if isinstance(v, np.ndarray) else v, inputs)
        elif isinstance(inputs, (np.ndarray, list)) and not isinstance(inputs, torch.Tensor):
            inputs = torch.as_tensor(np.asarray(inputs))
        return super().__call__(inputs, *args, **kwargs)

    # ------------------------------------------------------------ persistence
    def save(self, filepath, signatures=None, **kw):
        from .. import saved_model
        return saved_model.save(self, filepath, signatures=signatures)

    def save_weights(self, filepath):
        from ..train.checkpoint import Checkpoint
        return Checkpoint(model=self).write(filepath)

    def load_weights(self, filepath):
        from ..train.checkpoint import Checkpoint
        return Checkpoint(model=self).read(filepath)

    def get_weights(self):
        return [w.detach().cpu().numpy() for w in self.weights]

    def set_weights(self, values):
        for w, v in zip(self.weights, values):
            w.assign(torch.as_tensor(v))

    def summary(self, print_fn=print):
        print_fn(f'Model: "{self.name}"')
        print_fn(f"{'Layer':40s} {'Params':>12s}")
        for l in self.layers:
            print_fn(f"{l.name:40s} {l.count_params():>12,d}")
        print_fn(f"Total params: {self.count_params():,d}  "
                 f"(trainable {sum(w.numel() for w in self.trainable_weights):,d})")


class Sequential(Model):
    def __init__(self, layers=None, name=None, **kw):
        super().__init__(name=name, **kw)
        self._seq = []
        for l in layers or []:
            self.add(l)

    def add(self, layer):
        if isinstance(layer, (InputLayer, KL.KerasTensor)):
            self._input_shape = layer.input_shape
            return
        self._seq.append(layer)
        self._layers.append(layer)

    def build(self, input_shape=None):
        if input_shape is None and getattr(self, "_input_shape", None) is not None:
            input_shape = (1,) + tuple(self._input_shape)
        if input_shape is not None:
            dev = context.current_device()
            x = torch.zeros(input_shape, device=dev)
            with torch.no_grad():
                self.call(x, training=False)
        self.built = True

    def call(self, x, training=None):
        for l in self._seq:
            x = l(x, training=training)
        return x


def clone_model(model):
    return copy.deepcopy(model)


del time
