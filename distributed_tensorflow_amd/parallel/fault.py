"""Failure detection and fault injection (SURVEY §5 "Failure detection / elastic / fault injection").

The reference has nothing beyond the Supervisor's chief restore-on-start (reference trainer/task.py:215-226)
and swallows exceptions (:260-261). Here:
* ``Heartbeat``: a daemon thread that stamps ``hb/<task>`` in the coordination KV store every
  ``interval`` seconds; ``HeartbeatMonitor.dead(timeout)`` lists tasks whose stamp is stale.
* ``FaultInjector``: env-driven faults for tests (``DTF_FAULT``), e.g.
  ``kill@step=500`` (SIGKILL at training step 500), ``raise@step=10``, ``kill@ckpt=1`` (SIGKILL right
  after the first checkpoint is written), optionally restricted with ``@role=master0`` (matches
  ``DTF_ROLE``). A supervising launcher (cli.launch ``--max_restarts``) restarts the task without the
  fault, so "kill -9 the chief, then relaunch" runs unattended.
* ``retry``: re-run a closure on ConnectionError/TimeoutError (ClusterCoordinator rescheduling).
"""
from __future__ import annotations

import os
import signal
import threading
import time


class Heartbeat:
    """`kv` is any KVClient of the coordination service; the heartbeat opens its own connection to the
    same address (the native client is not shared across threads, and the owner may block in get())."""

    def __init__(self, kv, task, interval=1.0):
        from .kv import KVClient
        self.kv = KVClient(*kv.addr, timeout_s=30.0)
        self.task, self.interval = task, float(interval)
        self._stop = threading.Event()
        self._th = threading.Thread(target=self._run, daemon=True, name=f"heartbeat-{task}")
        self.beats = 0

    def start(self):
        self._beat()
        self._th.start()
        return self

    def _beat(self):
        self.kv.set(f"hb/{self.task}", repr(time.time()))
        self.beats += 1

    def _run(self):
        while not self._stop.wait(self.interval):
            try:
                self._beat()
            except Exception:  # coordination service gone: nothing left to report to
                return

    def stop(self):
        self._stop.set()
        if self._th.is_alive():
            self._th.join(timeout=2 * self.interval + 1)
        self.kv.close()


class HeartbeatMonitor:
    def __init__(self, kv, tasks):
        self.kv, self.tasks = kv, list(tasks)

    def last_seen(self, task):
        if not self.kv.check(f"hb/{task}"):
            return None
        return float(self.kv.get(f"hb/{task}", timeout_s=1.0))

    def dead(self, timeout=10.0, now=None):
        now = time.time() if now is None else now
        out = []
        for t in self.tasks:
            s = self.last_seen(t)
            if s is None or now - s > timeout:
                out.append(t)
        return out


class FaultInjector:
    def __init__(self, spec=None, role=None):
        spec = os.environ.get("DTF_FAULT", "") if spec is None else spec
        self.role = role if role is not None else os.environ.get("DTF_ROLE", "")
        self.action, self.trigger, self.at, self.only = None, None, None, None
        if spec:
            parts = spec.split("@")
            self.action = parts[0]
            for p in parts[1:]:
                k, _, v = p.partition("=")
                if k in ("step", "ckpt"):
                    self.trigger, self.at = k, int(v)
                elif k == "role":
                    self.only = v
            if self.action not in ("kill", "raise", "hang"):
                raise ValueError(f"bad DTF_FAULT action {self.action!r}")
        self.fired = False

    @property
    def armed(self):
        return self.action is not None and not self.fired and (self.only is None or self.only == self.role)

    def _fire(self, what):
        self.fired = True
        print(f"[fault] injecting {self.action} at {what} ({self.role})", flush=True)
        if self.action == "kill":
            os.kill(os.getpid(), signal.SIGKILL)
        elif self.action == "raise":
            raise RuntimeError(f"injected fault at {what}")
        else:
            while True:
                time.sleep(3600)

    def on_step(self, step):
        if self.armed and self.trigger == "step" and step >= self.at:
            self._fire(f"step {step}")

    def on_checkpoint(self, n_saved):
        if self.armed and self.trigger == "ckpt" and n_saved >= self.at:
            self._fire(f"checkpoint {n_saved}")


_global = None


def injector():
    global _global
    if _global is None:
        _global = FaultInjector()
    return _global


def retry(fn, *args, retries=3, backoff_s=0.5, exceptions=(ConnectionError, TimeoutError, OSError), **kwargs):
    for attempt in range(retries + 1):
        try:
            return fn(*args, **kwargs)
        except exceptions:
            if attempt == retries:
                raise
            time.sleep(backoff_s * (2 ** attempt))
