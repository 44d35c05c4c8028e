"""TensorBoard summaries: event files written by the native TFRecord/event writer.

TF1 surface used by the reference (trainer/task.py:72-74,80,92-98): ``FileWriter(logdir, graph)``,
``add_summary(summary, global_step)``, ``close()``, and scalar summaries tagged ``loss`` and
``training/hptuning/metric``. TF2 surface: ``create_file_writer(logdir).as_default()`` +
``scalar(name, value, step)`` / ``histogram`` / ``text``.
"""
from __future__ import annotations

import contextlib
import os
import socket
import struct
import threading
import time

import numpy as np

from .. import _native
from .._runtime_sigs import err

_default = threading.local()


def _event_path(logdir):
    os.makedirs(logdir, exist_ok=True)
    return os.path.join(logdir, f"events.out.tfevents.{int(time.time())}.{socket.gethostname()}.{os.getpid()}.v2")


def _varint(v):
    out = bytearray()
    while v >= 0x80:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)


def _field(num, wt, payload):
    return _varint(num << 3 | wt) + payload


def _ld(num, b):
    return _field(num, 2, _varint(len(b)) + b)


def histogram_proto(values, bins=30):
    v = np.asarray(values, dtype=np.float64).reshape(-1)
    if v.size == 0:
        v = np.zeros(1)
    counts, edges = np.histogram(v, bins=bins)
    h = b"".join([
        _field(1, 1, struct.pack("<d", float(v.min()))),
        _field(2, 1, struct.pack("<d", float(v.max()))),
        _field(3, 1, struct.pack("<d", float(v.size))),
        _field(4, 1, struct.pack("<d", float(v.sum()))),
        _field(5, 1, struct.pack("<d", float((v * v).sum()))),
        _ld(6, struct.pack(f"<{len(edges) - 1}d", *edges[1:])),
        _ld(7, struct.pack(f"<{len(counts)}d", *counts.astype(np.float64))),
    ])
    return h


def summary_value_histo(tag, values):
    return _ld(1, _ld(1, tag.encode()) + _ld(5, histogram_proto(values)))


def summary_value_scalar(tag, value):
    return _ld(1, _ld(1, tag.encode()) + _field(2, 5, struct.pack("<f", float(value))))


class SummaryWriter:
    def __init__(self, logdir):
        self.lib = _native.runtime()
        self.logdir = logdir
        self.path = _event_path(logdir)
        self.h = self.lib.dtfrt_events_open(self.path.encode())
        if not self.h:
            raise IOError(err(self.lib))
        self._lock = threading.Lock()

    def scalar(self, tag, value, step=0):
        v = float(value.item() if hasattr(value, "item") else value)
        with self._lock:
            self.lib.dtfrt_events_scalar(self.h, tag.encode(), v, int(step), 0.0)

    def histogram(self, tag, values, step=0):
        if hasattr(values, "detach"):
            values = values.detach().float().cpu().numpy()
        b = summary_value_histo(tag, values)
        with self._lock:
            self.lib.dtfrt_events_summary(self.h, b, len(b), int(step), 0.0)

    def text(self, tag, text, step=0):
        # Summary.Value.metadata.plugin_data.plugin_name = "text"; tensor string_val
        tensor = _field(1, 0, _varint(7)) + _ld(8, text.encode())
        meta = _ld(1, _ld(1, b"text"))
        b = _ld(1, _ld(1, tag.encode()) + _ld(9, meta) + _ld(8, tensor))
        with self._lock:
            self.lib.dtfrt_events_summary(self.h, b, len(b), int(step), 0.0)

    def add_summary(self, summary, global_step=0):
        """TF1 FileWriter.add_summary: bytes of a Summary proto, or a {tag: value} dict."""
        if isinstance(summary, dict):
            for k, v in summary.items():
                self.scalar(k, v, global_step)
        else:
            b = bytes(summary)
            with self._lock:
                self.lib.dtfrt_events_summary(self.h, b, len(b), int(global_step), 0.0)

    def add_graph(self, graph_description):
        b = graph_description.encode() if isinstance(graph_description, str) else bytes(graph_description)
        with self._lock:
            self.lib.dtfrt_events_graph(self.h, b, len(b), 0.0)

    def flush(self):
        with self._lock:
            if self.h:
                self.lib.dtfrt_tfrecord_flush(self.h)

    def close(self):
        with self._lock:
            if self.h:
                self.lib.dtfrt_tfrecord_writer_close(self.h)
                self.h = None

    @contextlib.contextmanager
    def as_default(self, step=None):
        prev = getattr(_default, "w", None)
        _default.w = self
        try:
            yield self
        finally:
            _default.w = prev
            self.flush()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def create_file_writer(logdir, **kw):
    return SummaryWriter(logdir)


def FileWriter(logdir, graph=None):
    """TF1 tf.summary.FileWriter(logdir, graph). `graph`: a serialized GraphDef, a graph_def.GraphBuilder, or a
    Model (its TF training graph, saved_model.graph_def.model_graph) — written as the Event.graph_def record that
    TensorBoard's graph dashboard renders."""
    w = SummaryWriter(logdir)
    if graph is not None:
        if hasattr(graph, "graph_def"):
            graph = graph.graph_def()
        elif hasattr(graph, "weights") and hasattr(graph, "trainable_variables"):
            from ..saved_model.graph_def import model_graph
            graph = model_graph(graph, training=True)[0].graph_def()
        w.add_graph(graph if isinstance(graph, (str, bytes)) else repr(graph))
    return w


_step = threading.local()


def experimental_set_step(step):
    _step.v = int(step)


def scalar(name, data, step=None):
    w = getattr(_default, "w", None)
    if w is None:
        return False
    w.scalar(name, data, step if step is not None else getattr(_step, "v", 0))
    return True


def histogram(name, data, step=None):
    w = getattr(_default, "w", None)
    if w is None:
        return False
    w.histogram(name, data, step if step is not None else getattr(_step, "v", 0))
    return True


def read_event_records(path):
    """The raw serialized Event protos of an event file, in order (TFRecord framing and CRCs checked)."""
    import ctypes
    lib = _native.runtime()
    h = lib.dtfrt_tfrecord_reader_open(path.encode())
    if not h:
        raise IOError(err(lib))
    out = []
    data = ctypes.c_void_p()
    n = ctypes.c_uint64()
    try:
        while True:
            rc = lib.dtfrt_tfrecord_next(h, ctypes.addressof(data), ctypes.addressof(n))
            if rc == 0:
                break
            if rc < 0:
                raise IOError(err(lib))
            out.append(ctypes.string_at(data.value, n.value))
    finally:
        lib.dtfrt_tfrecord_reader_close(h)
    return out


def read_events(path):
    """Parse an event file back into [(wall_time, step, {tag: value})] (used by tests and tooling)."""
    return [_parse_event(r) for r in read_event_records(path)]


def _read_varint(b, p):
    v, s = 0, 0
    while True:
        c = b[p]
        p += 1
        v |= (c & 0x7F) << s
        s += 7
        if not c & 0x80:
            return v, p


def _parse_fields(b):
    p = 0
    while p < len(b):
        k, p = _read_varint(b, p)
        f, wt = k >> 3, k & 7
        if wt == 0:
            v, p = _read_varint(b, p)
        elif wt == 1:
            v = b[p:p + 8]
            p += 8
        elif wt == 5:
            v = b[p:p + 4]
            p += 4
        elif wt == 2:
            ln, p = _read_varint(b, p)
            v = b[p:p + ln]
            p += ln
        else:
            raise ValueError("bad wire type")
        yield f, wt, v


def _parse_event(b):
    wall, step, vals = 0.0, 0, {}
    for f, wt, v in _parse_fields(b):
        if f == 1:
            wall = struct.unpack("<d", v)[0]
        elif f == 2:
            step = v
        elif f == 3:
            vals["__file_version__"] = v.decode()
        elif f == 5:
            for f2, _, val in _parse_fields(v):
                if f2 != 1:
                    continue
                tag, x = None, None
                for f3, _, y in _parse_fields(val):
                    if f3 == 1:
                        tag = y.decode()
                    elif f3 == 2:
                        x = struct.unpack("<f", y)[0]
                    elif f3 == 5:
                        x = "histogram"
                    elif f3 == 8:
                        x = "tensor"
                if tag is not None:
                    vals[tag] = x
    return wall, step, vals
