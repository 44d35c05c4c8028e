"""ManagedTraining: the tf.train.Supervisor lifecycle of the reference (trainer/task.py:215-226).

* chief: restore the latest checkpoint from ``logdir`` if there is one, else run the initializer;
  then a timer thread saves a checkpoint every ``save_model_secs`` (60 s in the reference) and a
  final checkpoint is written on exit;
* non-chief: wait until the chief has initialised the shared state (``wait_ready``), then train;
* ``global_step`` and the restored step are exposed so loops can resume where they stopped (the
  reference restarts its epoch loop at 0 after a restore — SURVEY Appendix A.5 — callers here can
  derive the epoch from the restored step).
Exceptions inside the managed block propagate (the reference swallowed them and exited 0,
SURVEY Appendix A.6).
"""
from __future__ import annotations

import os
import threading
import time

from .checkpoint import Saver, latest_checkpoint


class ManagedTraining:
    def __init__(self, is_chief, logdir, saver: Saver, global_step=None, init_fn=None, ready_fn=None,
                 save_model_secs=60, checkpoint_basename="model.ckpt", before_save=None):
        self.is_chief = is_chief
        self.logdir = logdir
        self.saver = saver
        self.global_step = global_step
        self.init_fn = init_fn
        self.ready_fn = ready_fn
        self.save_model_secs = save_model_secs
        self.base = checkpoint_basename
        self.before_save = before_save
        self.restored_from = None
        self._stop = threading.Event()
        self._th = None
        self._save_lock = threading.Lock()
        self.saves = 0

    def _step(self):
        gs = self.global_step
        if gs is None:
            return None
        return int(gs() if callable(gs) else gs.item())

    def save(self):
        with self._save_lock:
            if self.before_save is not None:
                self.before_save()
            p = self.saver.save(None, os.path.join(self.logdir, self.base), global_step=self._step())
            self.saves += 1
        from ..parallel.fault import injector
        injector().on_checkpoint(self.saves)  # DTF_FAULT=kill@ckpt=N (fault-tolerance tests)
        return p

    def _timer(self):
        while not self._stop.wait(self.save_model_secs):
            try:
                self.save()
            except Exception as e:  # keep training; report
                print(f"[supervisor] checkpoint failed: {e}", flush=True)

    def __enter__(self):
        if self.is_chief:
            os.makedirs(self.logdir, exist_ok=True)
            ck = latest_checkpoint(self.logdir)
            if ck:
                self.saver.restore(None, ck)
                self.restored_from = ck
            elif self.init_fn is not None:
                self.init_fn()
            if self.save_model_secs and self.save_model_secs > 0:
                self._th = threading.Thread(target=self._timer, daemon=True)
                self._th.start()
        elif self.ready_fn is not None:
            self.ready_fn()
        return self

    def should_stop(self):
        return self._stop.is_set()

    def request_stop(self):
        self._stop.set()

    def __exit__(self, exc_type, exc, tb):
        self._stop.set()
        if self._th is not None:
            self._th.join(timeout=30)
        if self.is_chief and exc_type is None:
            self.save()
        self.saver.wait()
        return False


del time
