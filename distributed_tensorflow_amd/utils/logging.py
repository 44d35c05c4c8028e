"""Rank-prefixed logging and a throughput meter.

The reference prints loss lines with ``print`` and its ``logging.info`` calls are invisible at the
default WARNING level. Here every process prefixes its role/rank and INFO is
visible by default (``DTF_LOG_LEVEL`` overrides).
"""
from __future__ import annotations

import logging as _logging
import os
import sys
import time

_configured = False


def get_logger(name="dtf", role=None):
    global _configured
    if not _configured:
        role = role or os.environ.get("DTF_ROLE") or f"rank{os.environ.get('RANK', '0')}"
        h = _logging.StreamHandler(sys.stdout)
        h.setFormatter(_logging.Formatter(f"[%(asctime)s {role} %(levelname)s] %(message)s", "%H:%M:%S"))
        root = _logging.getLogger("dtf")
        root.addHandler(h)
        root.setLevel(os.environ.get("DTF_LOG_LEVEL", "INFO"))
        root.propagate = False
        _configured = True
    return _logging.getLogger(name if name.startswith("dtf") else f"dtf.{name}")


class Throughput:
    """items/sec meter (images/sec, tokens/sec) over a window of steps."""

    def __init__(self):
        self.t0 = None
        self.items = 0
        self.steps = 0

    def start(self):
        self.t0 = time.perf_counter()
        self.items = self.steps = 0

    def step(self, n):
        self.items += n
        self.steps += 1

    def rate(self):
        dt = time.perf_counter() - self.t0
        return self.items / dt if dt > 0 else 0.0
