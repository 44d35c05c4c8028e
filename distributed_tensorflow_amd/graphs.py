"""hipGraph capture of training steps (the tf.function / XLA-free answer to per-op launch overhead).

``CapturedStep(fn)`` runs ``fn`` eagerly for ``warmup`` calls, then captures one call into
hipGraphs (``torch.cuda.CUDAGraph`` = hipGraph on ROCm) and afterwards only replays them: every HIP
kernel of forward, backward, gradient reduction and the fused optimizer update is issued by graph
launches, one per stream the step uses ("split" capture, the default): the main (data-gradient) stream's
graph, then the weight-gradient side stream's, then the communication stream's, each launched into its own
stream so the kernels keep the hardware queue and the overlap they have eagerly. Cross-stream edges become
external event nodes (earlier-launched graph -> later one) or bounded device-flag waits (the joins back into
main): csrc/kernels/graph_sync.hip. ``split=False`` (or torch.distributed process-group collectives in the
step) captures ONE multi-branch graph instead, whose branches the HIP runtime maps onto queues itself. Inputs are copied into static buffers; per-step scalars that the graph
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


SPLIT_DEFAULT = __import__("os").environ.get("DTF_GRAPH_SPLIT", "1") != "0"


class CapturedStep:
    def __init__(self, fn, warmup=2, optimizers=(), pool=None, split=None, static_inputs=False, require_split=False):
        self.fn = fn
        # require_split=True (multi-rank steps): capture only as per-stream graphs; when the step issues collectives
        # the per-stream capture cannot order (torch.distributed process-group Work objects), run eagerly instead of
        # capturing one multi-branch graph around them
        self.require_split = bool(require_split)
        self.eager = False
        # static_inputs=True: the caller promises that a replay argument which is the same tensor object as last
        # time, with an unchanged version counter, still holds the same values, so its copy into the static buffer is
        # skipped. Off by default: writes through .data, DLPack, numpy views of pinned staging buffers or native
        # kernels do not bump the version counter, and a skipped copy would then train on a stale batch.
        self.static_inputs = bool(static_inputs)
        self.warmup = warmup
        self.optimizers = list(optimizers)
        self.pool = pool
        self.split = SPLIT_DEFAULT if split is None else bool(split)
        self.graph = None
        self.sc = None        # ops._util.SplitCapture of a per-stream capture
        self.calls = 0
        self.static_in = None
        self.out = None
        self._errq = []  # (pinned copy of the capture's error flag, event after the copy) per replay in flight

    def _capture(self, args):
        from .ops import _util
        if self.require_split and not (self.split and _util.split_capture_ok()):
            self.eager = True
            return False
        flat = _flat(args, [])
        self.static_in = [t.clone() for t in flat]
        self._src = self._sources(flat)
        static_args = _rebuild(args, iter(self.static_in))
        for o in self.optimizers:
            o.graph_prepare()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        if self.split and _util.split_capture_ok():
            out = self._capture_split(g, static_args)
        else:
            self.sc = None
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
        return True

    def _capture_split(self, g, static_args):
        import gc
        from .ops import _util
        dev = torch.device("cuda", torch.cuda.current_device())
        pool = self.pool if self.pool is not None else torch.cuda.graph_pool_handle()
        self.pool = pool
        sc = _util.SplitCapture(dev, pool)
        cap = torch.cuda.Stream(device=dev)
        cap.wait_stream(torch.cuda.current_stream(dev))
        torch.cuda.synchronize()
        gc.collect()
        with torch.cuda.stream(cap):
            g.capture_begin(pool=pool, capture_error_mode="relaxed")
            ok = False
            try:
                sc.begin(cap)
                _util.set_split_capture(sc)
                out = self.fn(static_args)
                sc.finish()
                ok = True
            finally:
                _util.set_split_capture(None)
                if not ok:
                    sc.abort()
                g.capture_end()
        torch.cuda.current_stream(dev).wait_stream(cap)
        self.sc = sc
        return out

    @staticmethod
    def _sources(flat):
        import weakref
        out = []
        for t in flat:
            try:
                out.append((weakref.ref(t), t._version))
            except TypeError:
                out.append(None)
        return out

    def check(self):
        """Raise if a cross-stream flag wait of the per-stream graphs ever timed out (a broken edge; its replay's
        results are not to be trusted). Synchronises the device."""
        if self.sc is not None:
            e = int(self.sc.err.item())
            if e:
                raise RuntimeError(f"hipGraph per-stream replay: cross-stream wait {e - 1} timed out")

    ERR_DEPTH = 2  # replays the host may run ahead of the last error-flag check

    def _post_err_check(self):
        """Every replay copies the error flag to pinned memory behind an event; the copy of the replay ERR_DEPTH
        calls back is waited for and checked here. A timed-out cross-stream wait therefore raises within ERR_DEPTH
        replays (and the optimizer launches skipped their update since: ops.optim step_abort_ptr), while the host
        still runs up to ERR_DEPTH steps ahead of the GPU."""
        q = self._errq
        if len(q) >= self.ERR_DEPTH:
            buf, ev = q.pop(0)
            ev.synchronize()
            if int(buf[0]):
                raise RuntimeError(f"hipGraph per-stream replay: cross-stream wait {int(buf[0]) - 1} timed out; the "
                                   "step's optimizer update was skipped")
        else:
            buf, ev = torch.zeros(1, dtype=torch.int32).pin_memory(), torch.cuda.Event()
        buf.copy_(self.sc.err, non_blocking=True)
        ev.record()
        q.append((buf, ev))

    @property
    def captured(self):
        return self.graph is not None

    def __call__(self, args):
        self.calls += 1
        if self.eager:
            return self.fn(args)
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
            if not self._capture(args):
                return self.fn(args)
        else:
            flat = _flat(args, [])
            for i, (s, t) in enumerate(zip(self.static_in, flat)):
                # the very tensor whose contents the static buffer already holds (same object, no in-place write
                # since: torch's version counter, shared by its views): no copy (e.g. a fixed benchmark batch)
                src = self._src[i] if self.static_inputs else None
                if s.data_ptr() != t.data_ptr() and not (src is not None and src[0]() is t and t._version == src[1]):
                    s.copy_(t, non_blocking=True)
            if self.static_inputs:
                self._src = self._sources(flat)
        # per-step scalars go to a pinned ring (Optimizer.graph_prestep): no host sync between replays
        for o in self.optimizers:
            o.graph_prestep()
        self.graph.replay()
        if self.sc is not None:
            self.sc.replay_others()
            self._post_err_check()
        for o in self.optimizers:
            o.graph_poststep()
        from .ops import _util
        _util.bump_weights_epoch()
        return self._log_type(self.out) if self._log_type else self.out

    def reset(self):
        for o in self.optimizers:
            o._graph = None
        self.graph = None
        self.sc = None
        self.calls = 0
        self.eager = False
        self._errq = []


def function(fn=None, warmup=2, optimizers=(), split=None, static_inputs=False):
    """Decorator: ``@dtf.function`` captures a (static-shape) step into hipGraphs after `warmup` calls."""
    def wrap(f):
        return CapturedStep(f, warmup=warmup, optimizers=optimizers, split=split, static_inputs=static_inputs)
    return wrap(fn) if fn is not None else wrap
