"""Checkpoints in the TF tensor-bundle format (native writer/reader: csrc/runtime/tensor_bundle.cc).

* ``Saver`` — TF1 ``tf.train.Saver`` semantics used by the reference (trainer/task.py:143 plain,
  task_supervisor.py:145 ``sharded=True``): variables keyed by their names (``weight``, ``bias``,
  ``global_step``, optimizer slots ``weight/Adam``...), files ``model.ckpt-<step>.{index,data-*}``
  plus the ``checkpoint`` state file, ``max_to_keep`` rotation; sharded saves write one data file
  per PS shard.
* ``Checkpoint`` / ``CheckpointManager`` — TF2 object-based checkpoints
  (``<path>/.ATTRIBUTES/VARIABLE_VALUE`` keys) for Keras models and optimizers.
Saves are snapshot-then-write: device tensors are copied to host first (optionally on a side
stream), then a background thread writes the bundle, so training continues during the file IO.
"""
from __future__ import annotations

import ctypes
import json
import os
import re
import threading
import time

import numpy as np
import torch

from .. import _native
from .._runtime_sigs import err

_DT = {torch.float32: 1, torch.float64: 2, torch.int32: 3, torch.uint8: 4, torch.int16: 5, torch.int8: 6,
       torch.int64: 9, torch.bool: 10, torch.bfloat16: 14, torch.float16: 19}
_DT_INV = {v: k for k, v in _DT.items()}
DT_STRING = 7


class BundleWriter:
    def __init__(self, prefix, num_shards=1):
        self.lib = _native.runtime()
        d = os.path.dirname(prefix)
        if d:
            os.makedirs(d, exist_ok=True)
        self.h = self.lib.dtfrt_bundle_writer_open(prefix.encode(), int(num_shards))
        if not self.h:
            raise IOError(err(self.lib))
        self.prefix = prefix

    def add(self, name, tensor, shard=0):
        t = tensor.detach()
        if t.device.type != "cpu":
            t = t.cpu()
        t = t.contiguous()
        dims = (ctypes.c_int64 * max(1, t.dim()))(*t.shape)
        rc = self.lib.dtfrt_bundle_add(self.h, name.encode(), _DT[t.dtype], t.dim(), dims, t.data_ptr(),
                                       t.numel() * t.element_size(), int(shard))
        if rc:
            raise IOError(err(self.lib))

    def add_string(self, name, value, shard=0):
        b = value.encode() if isinstance(value, str) else bytes(value)
        arr = (ctypes.c_char_p * 1)(b)
        lens = (ctypes.c_int64 * 1)(len(b))
        dims = (ctypes.c_int64 * 1)(0)
        rc = self.lib.dtfrt_bundle_add_strings(self.h, name.encode(), 0, dims, 1, arr, lens, int(shard))
        if rc:
            raise IOError(err(self.lib))

    def finish(self):
        rc = self.lib.dtfrt_bundle_finish(self.h)
        self.h = None
        if rc:
            raise IOError(err(self.lib))
        return self.prefix


class BundleReader:
    def __init__(self, prefix):
        self.lib = _native.runtime()
        self.h = self.lib.dtfrt_bundle_reader_open(prefix.encode())
        if not self.h:
            raise IOError(err(self.lib))
        self.prefix = prefix

    def names(self):
        return [self.lib.dtfrt_bundle_name(self.h, i).decode() for i in range(self.lib.dtfrt_bundle_num_tensors(self.h))]

    def info(self, name):
        dt, nd, nb = ctypes.c_int(), ctypes.c_int(), ctypes.c_int64()
        dims = (ctypes.c_int64 * 16)()
        if self.lib.dtfrt_bundle_info(self.h, name.encode(), ctypes.addressof(dt), ctypes.addressof(nd), dims,
                                      ctypes.addressof(nb)):
            raise KeyError(name)
        return dt.value, tuple(dims[i] for i in range(nd.value)), nb.value

    def read(self, name):
        dt, shape, nb = self.info(name)
        buf = torch.empty(nb, dtype=torch.uint8)
        if self.lib.dtfrt_bundle_read(self.h, name.encode(), buf.data_ptr(), nb):
            raise IOError(err(self.lib))
        if dt == DT_STRING:
            return _decode_strings(buf.numpy().tobytes(), shape)
        return buf.view(_DT_INV[dt]).reshape(shape)

    def close(self):
        if self.h:
            self.lib.dtfrt_bundle_reader_close(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _decode_strings(b, shape):
    n = int(np.prod(shape)) if shape else 1
    lens, p = [], 0
    for _ in range(n):
        v, s = 0, 0
        while True:
            c = b[p]
            p += 1
            v |= (c & 0x7F) << s
            s += 7
            if not c & 0x80:
                break
        lens.append(v)
    p += 4  # masked crc of the length varints
    out = []
    for ln in lens:
        out.append(b[p:p + ln])
        p += ln
    return out[0] if not shape else out


def save_tensors(prefix, tensors, num_shards=1, shard_of=None):
    w = BundleWriter(prefix, num_shards)
    for i, (k, v) in enumerate(sorted(tensors.items())):
        if isinstance(v, (str, bytes)):
            w.add_string(k, v)
        else:
            w.add(k, torch.as_tensor(v), shard_of(k, i) if shard_of else 0)
    return w.finish()


def load_tensors(prefix):
    r = BundleReader(prefix)
    try:
        return {k: r.read(k) for k in r.names()}
    finally:
        r.close()


def list_variables(prefix):
    r = BundleReader(prefix)
    try:
        return [(k, list(r.info(k)[1])) for k in r.names()]
    finally:
        r.close()


def load_variable(prefix, name):
    r = BundleReader(prefix)
    try:
        return r.read(name)
    finally:
        r.close()


# ------------------------------------------------------------------ checkpoint state file
def _state_path(directory):
    return os.path.join(directory, "checkpoint")


def update_checkpoint_state(directory, model_checkpoint_path, all_paths):
    lines = [f'model_checkpoint_path: "{os.path.basename(model_checkpoint_path)}"']
    lines += [f'all_model_checkpoint_paths: "{os.path.basename(p)}"' for p in all_paths]
    tmp = _state_path(directory) + ".tmp"
    with open(tmp, "w") as f:
        f.write("\n".join(lines) + "\n")
    os.replace(tmp, _state_path(directory))


def get_checkpoint_state(directory):
    p = _state_path(directory)
    if not os.path.exists(p):
        return None
    model, allp = None, []
    for line in open(p):
        m = re.match(r'\s*(\w+):\s*"(.*)"', line)
        if not m:
            continue
        path = m.group(2)
        if not os.path.isabs(path):
            path = os.path.join(directory, path)
        if m.group(1) == "model_checkpoint_path":
            model = path
        elif m.group(1) == "all_model_checkpoint_paths":
            allp.append(path)
    return {"model_checkpoint_path": model, "all_model_checkpoint_paths": allp}


def latest_checkpoint(directory):
    st = get_checkpoint_state(directory)
    if st and st["model_checkpoint_path"] and os.path.exists(st["model_checkpoint_path"] + ".index"):
        return st["model_checkpoint_path"]
    return None


def _remove_checkpoint(prefix):
    d = os.path.dirname(prefix) or "."
    base = os.path.basename(prefix)
    for f in os.listdir(d):
        if f.startswith(base + ".index") or f.startswith(base + ".data-") or f == base + ".meta":
            try:
                os.remove(os.path.join(d, f))
            except OSError:
                pass


class _AsyncWriter:
    """Runs bundle writes on a background thread (one at a time, ordered)."""

    def __init__(self):
        self._th = None
        self._exc = None

    def submit(self, fn):
        self.wait()

        def run():
            try:
                fn()
            except Exception as e:  # surfaced at the next wait()
                self._exc = e
        self._th = threading.Thread(target=run, daemon=True)
        self._th.start()

    def wait(self):
        if self._th is not None:
            self._th.join()
            self._th = None
        if self._exc is not None:
            e, self._exc = self._exc, None
            raise e


def _snapshot(tensors):
    """Device -> host copies of every tensor (one sync at the end)."""
    out = {}
    for k, v in tensors.items():
        if isinstance(v, torch.Tensor):
            out[k] = v.detach().to("cpu", copy=True) if v.is_cuda else v.detach().clone()
        else:
            out[k] = v
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    return out


# ------------------------------------------------------------------ TF1 Saver
class Saver:
    """tf.train.Saver: name-keyed variables, optional sharding (one data file per PS shard)."""

    def __init__(self, var_list=None, sharded=False, num_shards=None, shard_of=None, max_to_keep=5,
                 async_write=False, meta_graph_def=None):
        """meta_graph_def: serialized MetaGraphDef (or a callable returning it) written as `<prefix>.meta` next to
        every checkpoint, like TF's Saver.save(write_meta_graph=True) (saved_model.graph_def.training_meta_graph)."""
        self.meta_graph_def = meta_graph_def
        if isinstance(var_list, dict):
            self.var_map = dict(var_list)
        else:
            self.var_map = {getattr(v, "name", f"var_{i}"): v for i, v in enumerate(var_list or [])}
        self.sharded = sharded
        self.num_shards = int(num_shards or (len(self.var_map) if sharded else 1)) if sharded else 1
        self.shard_of = shard_of
        self.max_to_keep = max_to_keep
        self._kept = []
        self._async = _AsyncWriter() if async_write else None

    def _shard(self, name, i):
        if not self.sharded:
            return 0
        if self.shard_of is not None:
            return int(self.shard_of(name)) % self.num_shards
        return i % self.num_shards

    def save(self, sess=None, save_path="model.ckpt", global_step=None, write_state=True, write_meta_graph=True):
        prefix = save_path if global_step is None else f"{save_path}-{int(_as_int(global_step))}"
        names = list(self.var_map)
        snap = _snapshot({k: self._value(v) for k, v in self.var_map.items()})
        meta = self.meta_graph_def() if callable(self.meta_graph_def) else self.meta_graph_def

        def write():
            w = BundleWriter(prefix, self.num_shards)
            for i, k in enumerate(names):
                w.add(k, snap[k], self._shard(k, i))
            w.finish()
            if write_meta_graph and meta:
                with open(prefix + ".meta.tmp", "wb") as f:
                    f.write(meta)
                os.replace(prefix + ".meta.tmp", prefix + ".meta")
            if write_state:
                d = os.path.dirname(prefix) or "."
                self._kept = [p for p in self._kept if p != prefix] + [prefix]
                while self.max_to_keep and len(self._kept) > self.max_to_keep:
                    _remove_checkpoint(self._kept.pop(0))
                update_checkpoint_state(d, prefix, self._kept)
        if self._async is not None:
            self._async.submit(write)
        else:
            write()
        return prefix

    def wait(self):
        if self._async is not None:
            self._async.wait()

    @staticmethod
    def _value(v):
        return v() if callable(v) and not isinstance(v, torch.Tensor) else v

    def restore(self, sess=None, save_path=None):
        r = BundleReader(save_path)
        try:
            have = set(r.names())
            for k, v in self.var_map.items():
                if k not in have:
                    raise KeyError(f"{k} not found in checkpoint {save_path}")
                t = r.read(k)
                _assign(v, t)
        finally:
            r.close()

    def recover_last_checkpoints(self, paths):
        self._kept = list(paths)


def _as_int(x):
    if isinstance(x, torch.Tensor):
        return int(x.item())
    return int(x)


def _assign(var, t):
    if hasattr(var, "assign"):
        var.assign(t.to(var.dtype).reshape(var.shape))
    else:
        with torch.no_grad():
            var.copy_(t.to(var.dtype).reshape(var.shape).to(var.device))


# ------------------------------------------------------------------ TF2 object checkpoints
_ATTR = "/.ATTRIBUTES/VARIABLE_VALUE"


def _collect(obj, path, out):
    """Flatten a trackable object tree into {key: tensor-like}."""
    from ..keras.layers import Layer
    from ..keras.optimizers import Optimizer
    if isinstance(obj, torch.Tensor):
        out[path + _ATTR] = obj
    elif isinstance(obj, Layer):
        for v in obj.weights:
            out[f"{path}/{v.name}{_ATTR}"] = v
    elif isinstance(obj, Optimizer):
        out[f"{path}/iter{_ATTR}"] = obj.iterations
        for a in obj._arenas.values():
            for nm in obj.get_slot_names():
                for v in a.variables:
                    out[f"{path}/slots/{v.name}/{nm}{_ATTR}"] = a.slot_view(nm, v)
    elif isinstance(obj, dict):
        for k, v in obj.items():
            _collect(v, f"{path}/{k}", out)
    elif isinstance(obj, (list, tuple)):
        for i, v in enumerate(obj):
            _collect(v, f"{path}/{i}", out)
    elif obj is not None:
        raise TypeError(f"cannot checkpoint {type(obj).__name__} at {path}")


class _RestoreStatus:
    def __init__(self, matched, missing, unused):
        self.matched, self.missing, self.unused = matched, missing, unused

    def assert_consumed(self):
        if self.missing or self.unused:
            raise AssertionError(f"missing={self.missing[:5]} unused={self.unused[:5]}")
        return self

    def assert_existing_objects_matched(self):
        if self.missing:
            raise AssertionError(f"missing={self.missing[:5]}")
        return self

    def expect_partial(self):
        return self


class Checkpoint:
    def __init__(self, **objects):
        from ..variables import Variable
        self._objects = objects
        self.save_counter = Variable(0, trainable=False, name="save_counter", dtype=torch.int64)
        self._async = _AsyncWriter()

    def _tensors(self):
        out = {}
        for k, v in self._objects.items():
            _collect(v, k, out)
        out["save_counter" + _ATTR] = self.save_counter
        return out

    def write(self, file_prefix, async_write=False, after=None):
        """Write the bundle; `after` (optional) runs once the bundle is complete (in the writer thread when
        asynchronous), e.g. to publish it in the `checkpoint` state file."""
        snap = _snapshot(self._tensors())
        meta = json.dumps({"keys": sorted(snap), "format": "dtf-object-graph-v1", "time": time.time()})

        def w():
            bw = BundleWriter(file_prefix)
            for k in sorted(snap):
                bw.add(k, snap[k])
            bw.add_string("_DTF_OBJECT_GRAPH_JSON", meta)
            bw.finish()
            if after is not None:
                after()
        if async_write:
            self._async.submit(w)
        else:
            w()
        return file_prefix

    MAX_STATE_PATHS = 100  # all_model_checkpoint_paths kept in the state file (most recent)

    def save(self, file_prefix, async_write=False):
        self.save_counter.assign_add(1)
        p = f"{file_prefix}-{int(self.save_counter.item())}"
        d = os.path.dirname(p) or "."

        def publish():  # only after the bundle is on disk: a crash mid-write keeps the previous good checkpoint
            st = get_checkpoint_state(d)
            allp = [q for q in (st["all_model_checkpoint_paths"] if st else []) if q != p] + [p]
            update_checkpoint_state(d, p, allp[-self.MAX_STATE_PATHS:])
        self.write(p, async_write, after=publish)
        return p

    def sync(self):
        self._async.wait()

    def read(self, save_path):
        self._async.wait()
        r = BundleReader(save_path)
        try:
            have = set(r.names()) - {"_DTF_OBJECT_GRAPH_JSON", "_CHECKPOINTABLE_OBJECT_GRAPH"}
            mine = self._tensors()
            matched, missing = [], []
            for k, v in mine.items():
                if k in have:
                    _assign(v, r.read(k))
                    matched.append(k)
                else:
                    missing.append(k)
            unused = sorted(have - set(mine))
        finally:
            r.close()
        from ..ops._util import bump_weights_epoch
        bump_weights_epoch()
        for obj in self._objects.values():
            if hasattr(obj, "reset_host_state"):
                obj.reset_host_state()
            for a in getattr(obj, "_arenas", {}).values():
                a.refresh_bf16()
        return _RestoreStatus(matched, missing, unused)

    restore = read


class CheckpointManager:
    def __init__(self, checkpoint, directory, max_to_keep=5, checkpoint_name="ckpt", keep_checkpoint_every_n_hours=None):
        self.checkpoint = checkpoint
        self.directory = directory
        self.max_to_keep = max_to_keep
        self.name = checkpoint_name
        os.makedirs(directory, exist_ok=True)
        st = get_checkpoint_state(directory)
        self._kept = [p for p in (st["all_model_checkpoint_paths"] if st else []) if os.path.exists(p + ".index")]

    @property
    def latest_checkpoint(self):
        return latest_checkpoint(self.directory)

    @property
    def checkpoints(self):
        return list(self._kept)

    def save(self, checkpoint_number=None, async_write=False):
        if checkpoint_number is None:
            self.checkpoint.save_counter.assign_add(1)
            checkpoint_number = int(self.checkpoint.save_counter.item())
        p = os.path.join(self.directory, f"{self.name}-{int(checkpoint_number)}")
        self.checkpoint.write(p, async_write=False)
        self._kept = [q for q in self._kept if q != p] + [p]
        while self.max_to_keep and len(self._kept) > self.max_to_keep:
            _remove_checkpoint(self._kept.pop(0))
        update_checkpoint_state(self.directory, p, self._kept)
        return p

    def restore_or_initialize(self):
        p = self.latest_checkpoint
        if p:
            self.checkpoint.restore(p)
        return p
