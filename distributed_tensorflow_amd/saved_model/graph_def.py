"""TF GraphDef / MetaGraphDef / SaverDef writer (hand-encoded protobuf wire format, no TF or protoc needed).

The reference exports a TF1 graph: the chief's ``SavedModelBuilder`` stores a MetaGraphDef holding the GraphDef of
the linear model (placeholders, ``weight``/``bias``/``global_step`` variables, Mul/Add), the internal Saver's
SaverDef and the ``serving_default`` SignatureDef (reference trainer/task.py:164-176, 275-289); ``FileWriter(path,
sess.graph)`` puts the GraphDef into the event file (trainer/task.py:80, 228) and the Supervisor's saver writes
``model.ckpt-N.meta`` next to every checkpoint [TF-RT]. This module builds those artifacts in TF's schemas
(tensorflow/core/framework/{graph,node_def,attr_value,tensor,tensor_shape,types}.proto and
tensorflow/core/protobuf/{meta_graph,saver}.proto) so a TF loader or TensorBoard can read them; the computation
itself still runs on this framework's kernels.

Names follow TF1 conventions: a variable ``v`` is the VariableV2 node ``v`` with ``v/initial_value`` (Const),
``v/Assign`` and the snapshot ``v/read``; the Saver subgraph is ``save/Const`` (the filename tensor),
``save/SaveV2`` + ``save/control_dependency`` (save tensor) and ``save/RestoreV2`` + ``save/Assign_*`` +
``save/restore_all`` (restore op), V2 (tensor-bundle) checkpoints.
"""
from __future__ import annotations

import struct

import numpy as np

DT = {"float32": 1, "float64": 2, "int32": 3, "uint8": 4, "string": 7, "int64": 9, "bool": 10, "bfloat16": 14,
      "float16": 19}
REF = 100  # DT_*_REF = DT_* + 100 (ref-typed outputs of VariableV2)
PRODUCER, MIN_CONSUMER = 27, 12  # VersionDef of a TF 1.x graph


# ---------------------------------------------------------------- protobuf wire helpers
def varint(v):
    v &= (1 << 64) - 1
    out = bytearray()
    while v >= 0x80:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)


def tag(f, wt):
    return varint(f << 3 | wt)


def ld(f, b):
    return tag(f, 2) + varint(len(b)) + b


def vi(f, v):
    return tag(f, 0) + varint(v)


def f32(f, v):
    return tag(f, 5) + struct.pack("<f", v)


def read_varint(b, p):
    v, s = 0, 0
    while True:
        c = b[p]
        p += 1
        v |= (c & 0x7F) << s
        s += 7
        if not c & 0x80:
            return v, p


def fields(b):
    """Decode one message level: yields (field number, value) with varints as ints, length-delimited as bytes."""
    p = 0
    while p < len(b):
        k, p = read_varint(b, p)
        f, wt = k >> 3, k & 7
        if wt == 0:
            v, p = read_varint(b, p)
        elif wt == 2:
            n, p = read_varint(b, p)
            v = bytes(b[p:p + n])
            p += n
        elif wt == 1:
            v = bytes(b[p:p + 8])
            p += 8
        elif wt == 5:
            v = bytes(b[p:p + 4])
            p += 4
        else:
            raise ValueError(f"bad wire type {wt}")
        yield f, v


# ---------------------------------------------------------------- schema pieces
def shape_proto(shape):
    """TensorShapeProto; None = unknown rank, -1 = unknown dim."""
    if shape is None:
        return vi(3, 1)
    return b"".join(ld(2, vi(1, int(d))) for d in shape)


def tensor_proto(value, dtype):
    """TensorProto of a numpy-convertible constant (tensor_content for numbers, string_val for strings)."""
    if dtype == "string":
        vals = value if isinstance(value, (list, tuple)) else [value]
        shape = [len(vals)] if isinstance(value, (list, tuple)) else []
        return vi(1, DT["string"]) + ld(2, shape_proto(shape)) + b"".join(
            ld(8, v if isinstance(v, bytes) else str(v).encode()) for v in vals)
    arr = np.asarray(value, dtype={"float32": np.float32, "float64": np.float64, "int32": np.int32,
                                   "int64": np.int64, "bool": np.bool_}[dtype])
    return vi(1, DT[dtype]) + ld(2, shape_proto(list(arr.shape))) + ld(4, arr.tobytes())


def attr_type(t):
    return vi(6, DT[t] if isinstance(t, str) else int(t))


def attr_shape(shape):
    return ld(7, shape_proto(shape))


def attr_tensor(value, dtype):
    return ld(8, tensor_proto(value, dtype))


def attr_bool(b):
    return vi(5, int(bool(b)))


def attr_int(i):
    return vi(3, int(i))


def attr_str(s):
    return ld(2, s if isinstance(s, bytes) else s.encode())


def attr_list_types(types):
    return ld(1, ld(6, b"".join(varint(DT[t]) for t in types)))


def attr_list_str(strs):
    return ld(1, b"".join(ld(2, s.encode()) for s in strs))


def _map_entry(f, key, value_bytes):
    return ld(f, ld(1, key.encode()) + ld(2, value_bytes))


# ---------------------------------------------------------------- graph builder
class GraphBuilder:
    """Accumulates NodeDefs; helpers for the op families the reference's graph uses."""

    def __init__(self):
        self.nodes = []      # (name, op, inputs, attrs dict)
        self._names = set()
        self.variables = []  # (name, dtype, shape, trainable)

    def unique(self, name):
        base, n = name, 1
        while name in self._names:
            name = f"{base}_{n}"
            n += 1
        return name

    def node(self, name, op, inputs=(), attrs=None, device=""):
        name = self.unique(name)
        self._names.add(name)
        self.nodes.append((name, op, list(inputs), dict(attrs or {}), device))
        return name

    # ---- op helpers (return the output tensor name "node:0" or node name for single-output ops)
    def placeholder(self, name, dtype, shape):
        return self.node(name, "Placeholder", (), {"dtype": attr_type(dtype), "shape": attr_shape(shape)})

    def const(self, name, value, dtype):
        return self.node(name, "Const", (), {"dtype": attr_type(dtype), "value": attr_tensor(value, dtype)})

    def identity(self, name, x, dtype):
        return self.node(name, "Identity", (x,), {"T": attr_type(dtype)})

    def binary(self, op, name, a, b, dtype="float32"):
        return self.node(name, op, (a, b), {"T": attr_type(dtype)})

    def unary(self, op, name, x, dtype="float32"):
        return self.node(name, op, (x,), {"T": attr_type(dtype)})

    def reduce_sum(self, name, x, rank, dtype="float32"):
        axes = self.const(f"{name}/reduction_indices", list(range(rank)), "int32")
        return self.node(name, "Sum", (x, axes), {"T": attr_type(dtype), "Tidx": attr_type("int32"),
                                                  "keep_dims": attr_bool(False)})

    def variable(self, name, value, dtype="float32", trainable=True):
        """VariableV2 + initial_value Const + Assign + read Identity; returns the read (snapshot) node."""
        arr = np.asarray(value)
        shape = list(arr.shape)
        v = self.node(name, "VariableV2", (), {"shape": attr_shape(shape), "dtype": attr_type(dtype),
                                                "container": attr_str(""), "shared_name": attr_str("")})
        init = self.const(f"{v}/initial_value", arr, dtype)
        self.node(f"{v}/Assign", "Assign", (v, init), {"T": attr_type(dtype), "validate_shape": attr_bool(True),
                                                       "use_locking": attr_bool(True),
                                                       "_class": attr_list_str([f"loc:@{v}"])})
        read = self.node(f"{v}/read", "Identity", (v,), {"T": attr_type(dtype), "_class": attr_list_str([f"loc:@{v}"])})
        self.variables.append((v, dtype, shape, trainable))
        return read

    def init_op(self, name="init"):
        return self.node(name, "NoOp", [f"^{v}/Assign" for v, _, _, _ in self.variables])

    def saver(self, prefix="save", max_to_keep=5, sharded=False):
        """The V2 Saver subgraph over every variable; returns the serialized SaverDef."""
        names = [v for v, _, _, _ in self.variables]
        dtypes = [d for _, d, _, _ in self.variables]
        fname = self.const(f"{prefix}/Const", "model", "string")
        tnames = self.const(f"{prefix}/SaveV2/tensor_names", names, "string")
        slices = self.const(f"{prefix}/SaveV2/shape_and_slices", [""] * len(names), "string")
        save = self.node(f"{prefix}/SaveV2", "SaveV2", [fname, tnames, slices] + names,
                         {"dtypes": attr_list_types(dtypes)})
        ctrl = self.node(f"{prefix}/control_dependency", "Identity", [fname, f"^{save}"],
                         {"T": attr_type("string"), "_class": attr_list_str([f"loc:@{fname}"])})
        rnames = self.const(f"{prefix}/RestoreV2/tensor_names", names, "string")
        rslices = self.const(f"{prefix}/RestoreV2/shape_and_slices", [""] * len(names), "string")
        restore = self.node(f"{prefix}/RestoreV2", "RestoreV2", [fname, rnames, rslices],
                            {"dtypes": attr_list_types(dtypes)})
        assigns = []
        for i, (v, d, _, _) in enumerate(self.variables):
            src = restore if i == 0 else f"{restore}:{i}"
            assigns.append(self.node(f"{prefix}/Assign", "Assign", (v, src),
                                     {"T": attr_type(d), "validate_shape": attr_bool(True),
                                      "use_locking": attr_bool(True), "_class": attr_list_str([f"loc:@{v}"])}))
        restore_all = self.node(f"{prefix}/restore_all", "NoOp", [f"^{a}" for a in assigns])
        return (ld(1, f"{fname}:0".encode()) + ld(2, f"{ctrl}:0".encode()) + ld(3, restore_all.encode()) +
                vi(4, max_to_keep) + vi(5, int(sharded)) + f32(6, 10000.0) + vi(7, 2))  # version V2

    # ---- serialization
    def graph_def(self):
        out = b""
        for name, op, inputs, attrs, device in self.nodes:
            nd = ld(1, name.encode()) + ld(2, op.encode()) + b"".join(ld(3, i.encode()) for i in inputs)
            if device:
                nd += ld(4, device.encode())
            for k in sorted(attrs):
                nd += _map_entry(5, k, attrs[k])
            out += ld(1, nd)
        return out + ld(4, vi(1, PRODUCER) + vi(2, MIN_CONSUMER))

    def variable_def(self, v):
        name, _, _, trainable = v
        return (ld(1, f"{name}:0".encode()) + ld(2, f"{name}/Assign".encode()) + ld(3, f"{name}/read:0".encode()) +
                ld(6, f"{name}/initial_value:0".encode()) + vi(7, int(trainable)))

    def collections(self, train_op=None):
        cols = {"variables": [self.variable_def(v) for v in self.variables],
                "trainable_variables": [self.variable_def(v) for v in self.variables if v[3]]}
        out = {}
        for k, vals in cols.items():
            if vals:
                out[k] = ld(2, b"".join(ld(1, b) for b in vals))  # CollectionDef.bytes_list
        if train_op:
            out["train_op"] = ld(1, ld(1, train_op.encode()))  # CollectionDef.node_list
        return out


def meta_graph_def(graph_def, tags=(), signature_defs=None, saver_def=None, collections=None):
    """Serialized MetaGraphDef."""
    info = ld(1, b"v1.0") + b"".join(ld(4, t.encode()) for t in tags) + ld(5, b"dtf (distributed_tensorflow_amd)")
    mg = ld(1, info) + ld(2, graph_def)
    if saver_def:
        mg += ld(3, saver_def)
    for k, v in sorted((collections or {}).items()):
        mg += _map_entry(4, k, v)
    for k, v in sorted((signature_defs or {}).items()):
        mg += _map_entry(5, k, v)
    return mg


# ---------------------------------------------------------------- decoding (tests, tooling)
def parse_graph_def(b):
    """-> list of {"name", "op", "input": [...], "attr": {key: raw AttrValue bytes}} and the VersionDef producer."""
    nodes, producer = [], None
    for f, v in fields(b):
        if f == 1:
            nd = {"name": "", "op": "", "input": [], "attr": {}, "device": ""}
            for f2, v2 in fields(v):
                if f2 == 1:
                    nd["name"] = v2.decode()
                elif f2 == 2:
                    nd["op"] = v2.decode()
                elif f2 == 3:
                    nd["input"].append(v2.decode())
                elif f2 == 4:
                    nd["device"] = v2.decode()
                elif f2 == 5:
                    key = val = None
                    for f3, v3 in fields(v2):
                        if f3 == 1:
                            key = v3.decode()
                        elif f3 == 2:
                            val = v3
                    nd["attr"][key] = val
            nodes.append(nd)
        elif f == 4:
            producer = dict(fields(v)).get(1)
    return nodes, producer


def parse_meta_graph(b):
    """-> {"tags", "graph_def" (bytes), "saver_def" {filename_tensor_name, save_tensor_name, restore_op_name,
    version}, "collections" {name: raw}, "signatures" {key: raw}}."""
    out = {"tags": [], "graph_def": b"", "saver_def": None, "collections": {}, "signatures": {}}
    for f, v in fields(b):
        if f == 1:
            out["tags"] = [v2.decode() for f2, v2 in fields(v) if f2 == 4]
        elif f == 2:
            out["graph_def"] = v
        elif f == 3:
            sd = {}
            names = {1: "filename_tensor_name", 2: "save_tensor_name", 3: "restore_op_name"}
            for f2, v2 in fields(v):
                if f2 in names:
                    sd[names[f2]] = v2.decode()
                elif f2 == 7:
                    sd["version"] = v2
                elif f2 == 4:
                    sd["max_to_keep"] = v2
            out["saver_def"] = sd
        elif f in (4, 5):
            key = val = None
            for f2, v2 in fields(v):
                if f2 == 1:
                    key = v2.decode()
                elif f2 == 2:
                    val = v2
            out["collections" if f == 4 else "signatures"][key] = val
    return out


def attr_value_type(raw):
    """DataType enum of an AttrValue holding a type (or None)."""
    return dict(fields(raw)).get(6)


# ---------------------------------------------------------------- model graphs
def variables_graph(model, builder=None):
    """VariableV2 nodes (+ initializers) for every weight of `model` (TF names: '/' separated scopes)."""
    g = builder or GraphBuilder()
    reads = {}
    for v in model.weights:
        arr = v.detach().float().cpu().numpy() if v.dtype.is_floating_point else v.detach().cpu().numpy()
        dt = "float32" if v.dtype.is_floating_point else ("int64" if str(v.dtype) == "torch.int64" else "int32")
        reads[v.name] = g.variable(v.name, arr.astype(np.float32 if dt == "float32" else
                                                      (np.int64 if dt == "int64" else np.int32)), dt,
                                   trainable=getattr(v, "trainable", True))
    return g, reads


def model_graph(model, training=False, optimizer=None):
    """GraphBuilder holding `model`'s TF graph: the model's own computation when it provides ``tf_graph(builder,
    reads, training, optimizer)`` (the reference's linear model does), otherwise its variables (+ init op).
    Returns (builder, signature tensor names or None, train_op name or None)."""
    g, reads = variables_graph(model)
    names = train_op = None
    if hasattr(model, "tf_graph"):
        names, train_op = model.tf_graph(g, reads, training=training,
                                         optimizer=optimizer if optimizer is not None else
                                         getattr(model, "optimizer", None))
    g.init_op()
    return g, names, train_op


def training_meta_graph(model, optimizer=None, tags=()):
    """The MetaGraphDef a TF1 Saver writes next to a checkpoint (``model.ckpt-N.meta``): the training graph, its
    SaverDef and the variables / trainable_variables / train_op collections."""
    g, _, train_op = model_graph(model, training=True, optimizer=optimizer)
    saver = g.saver()
    return meta_graph_def(g.graph_def(), tags=tags, saver_def=saver, collections=g.collections(train_op))
