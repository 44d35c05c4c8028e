"""SavedModel export / load.

Layout (reference trainer/task.py:264-291 writes ``saved_model_path/<model_version>/``):
  <dir>/saved_model.pb            SavedModel protobuf (schema of tensorflow/core/protobuf/saved_model.proto,
                                  hand-encoded): one MetaGraphDef tagged ``serve`` whose signature_def map
                                  holds ``serving_default`` (method ``tensorflow/serving/predict``)
  <dir>/variables/variables.{index,data-00000-of-00001}   tensor bundle (native writer)
  <dir>/dtf_model.json            how to rebuild the computation in this framework (class + init args +
                                  build shape + signature -> method): this framework runs the model on its
                                  own kernels. The MetaGraphDef also holds a real TF GraphDef (graph_def.py):
                                  every variable as VariableV2 + initializer, the V2 Saver subgraph and its
                                  SaverDef, the variables collections, and — for models that describe their
                                  computation (the reference's linear model: Placeholder, Identity, Mul,
                                  Add) — the serving graph whose tensors the signature names.
The reference's legacy ``session_bundle`` exporter (trainer/task.py:294-307) is superseded by this
format.
"""
from __future__ import annotations

import importlib
import json
import os
import struct

import torch

from ..train.checkpoint import BundleReader, BundleWriter

SERVING = "serve"
DEFAULT_SERVING_SIGNATURE_DEF_KEY = "serving_default"
PREDICT_METHOD_NAME = "tensorflow/serving/predict"
_DT = {"float32": 1, "float64": 2, "int32": 3, "uint8": 4, "int64": 9, "bool": 10, "bfloat16": 14, "string": 7,
       "float16": 19}
_DT_INV = {v: k for k, v in _DT.items()}


# ---------------------------------------------------------------- protobuf wire helpers
def _varint(v):
    v &= (1 << 64) - 1
    out = bytearray()
    while v >= 0x80:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)


def _tag(f, wt):
    return _varint(f << 3 | wt)


def _ld(f, b):
    return _tag(f, 2) + _varint(len(b)) + b


def _vi(f, v):
    return _tag(f, 0) + _varint(v)


def _shape_proto(shape):
    return b"".join(_ld(2, _vi(1, d)) for d in shape)


def _tensor_info(name, dtype, shape):
    return _ld(1, name.encode()) + _vi(2, _DT[dtype]) + _ld(3, _shape_proto(shape))


def _map_entry(f, key, value_bytes):
    return _ld(f, _ld(1, key.encode()) + _ld(2, value_bytes))


def signature_def(inputs, outputs, method_name=PREDICT_METHOD_NAME, tensor_names=None):
    """inputs/outputs: {key: (dtype, shape)} -> serialized SignatureDef. tensor_names: {"inputs": {key: "node:0"},
    "outputs": {...}} — the graph tensors the keys bind to (default "<key>:0")."""
    tn = tensor_names or {}
    b = b""
    for k, (dt, shp) in sorted(inputs.items()):
        b += _map_entry(1, k, _tensor_info(tn.get("inputs", {}).get(k, f"{k}:0"), dt, shp))
    for k, (dt, shp) in sorted(outputs.items()):
        b += _map_entry(2, k, _tensor_info(tn.get("outputs", {}).get(k, f"{k}:0"), dt, shp))
    b += _ld(3, method_name.encode())
    return b


def saved_model_proto(signatures, tags=(SERVING,), graph_def=b"", saver_def=None, collections=None):
    from .graph_def import meta_graph_def
    mg = meta_graph_def(graph_def, tags=tags, signature_defs=signatures, saver_def=saver_def,
                        collections=collections)
    return _vi(1, 1) + _ld(2, mg)


def _read_varint(b, p):
    v, s = 0, 0
    while True:
        c = b[p]
        p += 1
        v |= (c & 0x7F) << s
        s += 7
        if not c & 0x80:
            return v, p


def _fields(b):
    p = 0
    while p < len(b):
        k, p = _read_varint(b, p)
        f, wt = k >> 3, k & 7
        if wt == 0:
            v, p = _read_varint(b, p)
        elif wt == 2:
            n, p = _read_varint(b, p)
            v = b[p:p + n]
            p += n
        elif wt == 1:
            v = b[p:p + 8]
            p += 8
        elif wt == 5:
            v = b[p:p + 4]
            p += 4
        else:
            raise ValueError("bad wire type")
        yield f, v


def parse_saved_model(b):
    """-> {"tags": [...], "signatures": {key: {"inputs": {k: (dtype, shape)}, "outputs": ..., "method_name"}}}"""
    out = {"meta_graphs": []}
    for f, v in _fields(b):
        if f != 2:
            continue
        mg = {"tags": [], "signatures": {}}
        for f2, v2 in _fields(v):
            if f2 == 1:
                for f3, v3 in _fields(v2):
                    if f3 == 4:
                        mg["tags"].append(v3.decode())
            elif f2 == 5:
                key, sig = None, None
                for f3, v3 in _fields(v2):
                    if f3 == 1:
                        key = v3.decode()
                    elif f3 == 2:
                        sig = _parse_sig(v3)
                mg["signatures"][key] = sig
        out["meta_graphs"].append(mg)
    return out


def _parse_sig(b):
    sig = {"inputs": {}, "outputs": {}, "method_name": ""}
    for f, v in _fields(b):
        if f in (1, 2):
            key, ti = None, None
            for f2, v2 in _fields(v):
                if f2 == 1:
                    key = v2.decode()
                elif f2 == 2:
                    dt, shape, name = None, [], None
                    for f3, v3 in _fields(v2):
                        if f3 == 1:
                            name = v3.decode()
                        elif f3 == 2:
                            dt = _DT_INV.get(v3, str(v3))
                        elif f3 == 3:
                            for f4, v4 in _fields(v3):
                                if f4 == 2:
                                    for f5, v5 in _fields(v4):
                                        if f5 == 1:
                                            shape.append(v5 - (1 << 64) if v5 >= 1 << 63 else v5)
                    ti = (dt, shape)
            sig["inputs" if f == 1 else "outputs"][key] = ti
        elif f == 3:
            sig["method_name"] = v.decode()
    return sig


# ---------------------------------------------------------------- layer (de)serialization
def serialize_object(obj):
    from ..keras.layers import Layer
    if isinstance(obj, Layer):
        args, kwargs = getattr(obj, "_init_args", ((), {}))
        if hasattr(obj, "_seq"):  # Sequential: layers added after construction count too
            args, kwargs = (list(obj._seq),), {"name": obj.name}
        return {"__layer__": f"{type(obj).__module__}.{type(obj).__qualname__}",
                "args": [serialize_object(a) for a in args],
                "kwargs": {k: serialize_object(v) for k, v in kwargs.items()}}
    if isinstance(obj, (list, tuple)):
        return {"__seq__": type(obj).__name__, "items": [serialize_object(o) for o in obj]}
    if isinstance(obj, dict):
        return {"__dict__": {k: serialize_object(v) for k, v in obj.items()}}
    if obj is None or isinstance(obj, (int, float, str, bool)):
        return obj
    raise TypeError(f"cannot serialize {type(obj).__name__} into dtf_model.json")


def deserialize_object(d):
    if isinstance(d, dict):
        if "__layer__" in d:
            mod, _, name = d["__layer__"].rpartition(".")
            cls = getattr(importlib.import_module(mod), name)
            return cls(*[deserialize_object(a) for a in d["args"]],
                       **{k: deserialize_object(v) for k, v in d["kwargs"].items()})
        if "__seq__" in d:
            items = [deserialize_object(o) for o in d["items"]]
            return tuple(items) if d["__seq__"] == "tuple" else items
        if "__dict__" in d:
            return {k: deserialize_object(v) for k, v in d["__dict__"].items()}
    return d


def _default_signature(model):
    shp = getattr(model, "_build_input_shape", None)
    if shp is None:
        raise ValueError("model is not built; call it once or pass signatures=")
    return {"inputs": {"inputs": ("float32", [-1] + list(shp[1:]))},
            "outputs": {"outputs": ("float32", [-1])}, "method_name": PREDICT_METHOD_NAME, "fn": "__call__"}


def save(model, export_dir, signatures=None):
    """Export `model` as a SavedModel directory (chief-only in distributed training)."""
    os.makedirs(os.path.join(export_dir, "variables"), exist_ok=True)
    sig = signatures or (model.serving_signature() if hasattr(model, "serving_signature") else
                         _default_signature(model))
    from .graph_def import model_graph
    g, tensor_names, _ = model_graph(model, training=False)
    saver_def = g.saver()
    sig_defs = {DEFAULT_SERVING_SIGNATURE_DEF_KEY: signature_def(sig["inputs"], sig["outputs"],
                                                                 sig.get("method_name", PREDICT_METHOD_NAME),
                                                                 tensor_names)}
    w = BundleWriter(os.path.join(export_dir, "variables", "variables"))
    for v in model.weights:
        w.add(v.name, v.detach())
    w.finish()
    spec = {"format": "dtf-saved-model-v1", "model": serialize_object(model),
            "build_input_shape": list(getattr(model, "_build_input_shape", None) or []) or None,
            "signatures": {DEFAULT_SERVING_SIGNATURE_DEF_KEY: sig},
            "variables": [v.name for v in model.weights]}
    with open(os.path.join(export_dir, "dtf_model.json"), "w") as f:
        json.dump(spec, f, indent=1)
    tmp = os.path.join(export_dir, "saved_model.pb.tmp")
    with open(tmp, "wb") as f:
        f.write(saved_model_proto(sig_defs, graph_def=g.graph_def(), saver_def=saver_def,
                                  collections=g.collections()))
    os.replace(tmp, os.path.join(export_dir, "saved_model.pb"))
    return export_dir


_TORCH_DT = {"float32": torch.float32, "float64": torch.float64, "int32": torch.int32, "int64": torch.int64,
             "bool": torch.bool, "uint8": torch.uint8, "bfloat16": torch.bfloat16, "float16": torch.float16}


class _Signature:
    def __init__(self, model, spec):
        self.model = model
        self.spec = spec
        self.structured_input_signature = spec["inputs"]
        self.structured_outputs = spec["outputs"]

    def coerce(self, **inputs):
        """Cast JSON-ish inputs to the signature's dtypes (the README request sends keys as floats)."""
        out = {}
        dev = next(iter(self.model.weights)).device if self.model.weights else torch.device("cpu")
        for k, (dt, shp) in self.spec["inputs"].items():
            if k not in inputs:
                raise KeyError(f"missing input {k!r}")
            t = torch.as_tensor(inputs[k]) if not isinstance(inputs[k], torch.Tensor) else inputs[k]
            tdt = _TORCH_DT[dt]
            if not tdt.is_floating_point and t.is_floating_point():
                t = t.round()
            t = t.to(tdt)
            if len(shp) == 2 and t.dim() == 1:
                t = t.reshape(-1, 1)
            out[k] = t.to(dev)
        return out

    def __call__(self, **inputs):
        x = self.coerce(**inputs)
        fn = self.spec.get("fn", "__call__")
        with torch.no_grad():
            if fn == "__call__":
                (only,) = x.values()
                res = self.model(only, training=False)
                res = {next(iter(self.spec["outputs"])): res}
            else:
                res = getattr(self.model, fn)(**x)
        return {k: v for k, v in res.items()}


class Loaded:
    def __init__(self, model, signatures, tags):
        self.model = model
        self.signatures = signatures
        self.tags = tags

    def __call__(self, *a, **k):
        return self.model(*a, **k)


def load(export_dir, tags=None, device=None):
    from .. import context
    with open(os.path.join(export_dir, "saved_model.pb"), "rb") as f:
        pb = parse_saved_model(f.read())
    with open(os.path.join(export_dir, "dtf_model.json")) as f:
        spec = json.load(f)
    dev = context.parse_device(device) if device is not None else torch.device("cpu")
    with context.device(dev):
        model = deserialize_object(spec["model"])
        shp = spec.get("build_input_shape")
        if shp and not model.built:
            with torch.no_grad():
                model(torch.zeros([1] + list(shp[1:]), device=dev), training=False)
    r = BundleReader(os.path.join(export_dir, "variables", "variables"))
    try:
        have = set(r.names())
        for v in model.weights:
            if v.name in have:
                v.assign(r.read(v.name).reshape(v.shape))
    finally:
        r.close()
    sigs = {k: _Signature(model, s) for k, s in spec["signatures"].items()}
    return Loaded(model, sigs, pb["meta_graphs"][0]["tags"] if pb["meta_graphs"] else [])


def latest_version_dir(base):
    """simple_tensorflow_serving / TF-Serving convention: highest integer subdirectory."""
    vs = [int(d) for d in os.listdir(base) if d.isdigit() and os.path.isdir(os.path.join(base, d))]
    if not vs:
        if os.path.exists(os.path.join(base, "saved_model.pb")):
            return base
        raise FileNotFoundError(f"no model versions under {base}")
    return os.path.join(base, str(max(vs)))


del struct
