"""MonitoredTrainingSession + SessionRunHooks (tf.compat.v1.train surface).

The reference keeps a ``MonitoredTrainingSession(is_chief, checkpoint_dir, hooks=[StopAtStepHook(1e6)])``
loop inside a string literal (reference trainer/task.py:178-213). This module makes that
path real on our runtime: the session is a context manager that (chief) restores the latest checkpoint
from ``checkpoint_dir``, runs default chief hooks (timed CheckpointSaverHook, StepCounterHook writing
``global_step/sec``, SummarySaverHook) plus user hooks around every ``run(step_fn, ...)`` call, and
reports ``should_stop()`` once a hook requests it. ``run`` takes a Python step function (e.g.
``model.train_step``) instead of graph fetches; hooks see its return value as ``run_values.results``.
"""
from __future__ import annotations

import math
import os
import time

from .checkpoint import Saver, latest_checkpoint


class SessionRunContext:
    def __init__(self, session, args):
        self.session = session
        self.original_args = args
        self._stop = False

    def request_stop(self):
        self._stop = True

    @property
    def stop_requested(self):
        return self._stop


class SessionRunValues:
    def __init__(self, results):
        self.results = results


class SessionRunHook:
    def begin(self): pass
    def after_create_session(self, session, coord=None): pass
    def before_run(self, run_context): return None
    def after_run(self, run_context, run_values): pass
    def end(self, session): pass


class StopAtStepHook(SessionRunHook):
    """Stop at ``last_step`` (absolute) or after ``num_steps`` more steps."""

    def __init__(self, num_steps=None, last_step=None):
        if (num_steps is None) == (last_step is None):
            raise ValueError("exactly one of num_steps / last_step")
        self.num_steps, self.last_step = num_steps, last_step

    def after_create_session(self, session, coord=None):
        if self.last_step is None:
            self.last_step = session.global_step + int(self.num_steps)

    def after_run(self, run_context, run_values):
        if run_context.session.global_step >= self.last_step:
            run_context.request_stop()


class CheckpointSaverHook(SessionRunHook):
    def __init__(self, checkpoint_dir, save_secs=None, save_steps=None, saver=None,
                 checkpoint_basename="model.ckpt"):
        if save_secs is None and save_steps is None:
            save_secs = 600
        self.dir, self.save_secs, self.save_steps = checkpoint_dir, save_secs, save_steps
        self.saver, self.base = saver, checkpoint_basename
        self._last_t = time.time()
        self._last_step = None
        self.saves = 0

    def _save(self, session):
        if self.saver is None:
            return
        os.makedirs(self.dir, exist_ok=True)
        self.saver.save(None, os.path.join(self.dir, self.base), global_step=session.global_step)
        self._last_t, self._last_step = time.time(), session.global_step
        self.saves += 1

    def after_create_session(self, session, coord=None):
        self._last_step = session.global_step

    def after_run(self, run_context, run_values):
        s = run_context.session
        due = (self.save_secs is not None and time.time() - self._last_t >= self.save_secs) or (
            self.save_steps is not None and s.global_step - (self._last_step or 0) >= self.save_steps)
        if due:
            self._save(s)

    def end(self, session):
        if session.global_step != self._last_step:
            self._save(session)


class StepCounterHook(SessionRunHook):
    """Writes ``global_step/sec`` every N steps (the Supervisor's SVStepCounterThread)."""

    def __init__(self, every_n_steps=100, output_dir=None, summary_writer=None):
        self.every, self.dir, self.writer = every_n_steps, output_dir, summary_writer
        self._t, self._s = None, None
        self.rates = []

    def begin(self):
        if self.writer is None and self.dir is not None:
            from ..summary import FileWriter
            self.writer = FileWriter(self.dir)

    def after_run(self, run_context, run_values):
        gs = run_context.session.global_step
        now = time.time()
        if self._t is None:
            self._t, self._s = now, gs
            return
        if gs - self._s >= self.every:
            rate = (gs - self._s) / max(now - self._t, 1e-9)
            self.rates.append(rate)
            if self.writer is not None:
                self.writer.add_summary({"global_step/sec": rate}, gs)
            self._t, self._s = now, gs

    def end(self, session):
        if self.writer is not None and self.dir is not None:
            self.writer.close()


class SummarySaverHook(SessionRunHook):
    """Every ``save_steps``: write the scalars returned by ``scalars_fn(results)`` (or the float
    entries of a logs dict) at the current global step."""

    def __init__(self, save_steps=100, output_dir=None, summary_writer=None, scalars_fn=None):
        self.every, self.dir, self.writer, self.fn = save_steps, output_dir, summary_writer, scalars_fn

    def begin(self):
        if self.writer is None and self.dir is not None:
            from ..summary import FileWriter
            self.writer = FileWriter(self.dir)

    def after_run(self, run_context, run_values):
        gs = run_context.session.global_step
        if self.writer is None or gs % self.every:
            return
        res = run_values.results
        vals = self.fn(res) if self.fn else {k: float(v) for k, v in (res.items() if hasattr(res, "items") else [])}
        if vals:
            self.writer.add_summary(vals, gs)

    def end(self, session):
        if self.writer is not None and self.dir is not None:
            self.writer.close()


class LoggingTensorHook(SessionRunHook):
    def __init__(self, tensors, every_n_iter=100, formatter=None):
        self.tensors, self.every, self.fmt = tensors, every_n_iter, formatter
        self._n = 0
        self.lines = []

    def after_run(self, run_context, run_values):
        self._n += 1
        if self._n % self.every:
            return
        vals = {k: (f(run_values.results) if callable(f) else run_values.results[f]) for k, f in self.tensors.items()}
        line = self.fmt(vals) if self.fmt else ", ".join(f"{k} = {float(v):.6g}" for k, v in vals.items())
        self.lines.append(line)
        print(line, flush=True)


class NanTensorHook(SessionRunHook):
    def __init__(self, loss_fn=lambda r: r["loss"], fail_on_nan_loss=True):
        self.loss_fn, self.fail = loss_fn, fail_on_nan_loss

    def after_run(self, run_context, run_values):
        v = float(self.loss_fn(run_values.results))
        if math.isnan(v) or math.isinf(v):
            if self.fail:
                raise FloatingPointError("NaN loss during training")
            run_context.request_stop()


class MonitoredTrainingSession:
    """with MonitoredTrainingSession(is_chief, checkpoint_dir, variables=..., hooks=[...]) as sess:
           while not sess.should_stop():
               sess.run(model.train_step, batch)

    ``global_step`` counts ``run`` calls (resumed from the restored checkpoint's ``global_step``);
    pass ``global_step_fn`` to read it from elsewhere (e.g. the PS's shared counter)."""

    def __init__(self, is_chief=True, checkpoint_dir=None, variables=None, hooks=None, chief_only_hooks=None,
                 save_checkpoint_secs=600, save_checkpoint_steps=None, save_summaries_steps=100,
                 log_step_count_steps=100, global_step_fn=None, saver=None):
        self.is_chief = is_chief
        self.dir = checkpoint_dir
        self.variables = variables or {}
        self.saver = saver or (Saver(self.variables) if self.variables else None)
        self._gs_fn = global_step_fn
        self._gs = 0
        self._stop = False
        self.hooks = list(hooks or [])
        if is_chief:
            self.hooks += list(chief_only_hooks or [])
            if checkpoint_dir and (save_checkpoint_secs or save_checkpoint_steps) and self.saver is not None:
                self.hooks.append(CheckpointSaverHook(checkpoint_dir, save_checkpoint_secs, save_checkpoint_steps,
                                                      self.saver))
            if checkpoint_dir and log_step_count_steps:
                self.hooks.append(StepCounterHook(log_step_count_steps, checkpoint_dir))
        self.restored_from = None

    @property
    def global_step(self):
        return int(self._gs_fn()) if self._gs_fn is not None else self._gs

    def __enter__(self):
        for h in self.hooks:
            h.begin()
        if self.is_chief and self.dir and self.saver is not None:
            ck = latest_checkpoint(self.dir)
            if ck:
                self.saver.restore(None, ck)
                self.restored_from = ck
                gsv = self.variables.get("global_step")
                if gsv is not None:
                    self._gs = int(gsv.item())
        for h in self.hooks:
            h.after_create_session(self, None)
        return self

    def run(self, fn, *args, **kwargs):
        if self._stop:
            raise RuntimeError("run() called after should_stop()")
        ctx = SessionRunContext(self, (args, kwargs))
        for h in self.hooks:
            h.before_run(ctx)
        res = fn(*args, **kwargs)
        self._gs += 1
        gsv = self.variables.get("global_step")
        if gsv is not None and self._gs_fn is None:
            gsv.fill_(self._gs)
        vals = SessionRunValues(res)
        for h in self.hooks:
            h.after_run(ctx, vals)
        if ctx.stop_requested:
            self._stop = True
        return res

    def should_stop(self):
        return self._stop

    def request_stop(self):
        self._stop = True

    def __exit__(self, et, ev, tb):
        if et is None:
            for h in self.hooks:
                h.end(self)
        return False
