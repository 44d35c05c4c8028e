"""TF-compatible artifacts, checked structurally (TF itself is not importable here: parity unpinned).

The GraphDef / MetaGraphDef / SaverDef / SavedModel bytes this framework writes are parsed with the protobuf
runtime against message classes built from TF's own schema (field numbers and types of graph.proto,
node_def.proto, attr_value.proto, tensor.proto, meta_graph.proto, saver.proto, saved_model.proto, event.proto),
so a field-number or wire-type mistake fails here the way it would in a TF loader. Reference call sites:
trainer/task.py:80,228 (graph event), :164-176,275-289 (SavedModel with serving_default), :215-223 (Supervisor
checkpoints, whose Saver writes model.ckpt-N.meta).
"""
import glob
import os

import numpy as np
import pytest
import torch

from distributed_tensorflow_amd.saved_model import graph_def as GD


def _tf_schema():
    from google.protobuf import descriptor_pb2, descriptor_pool, message_factory
    F = descriptor_pb2.FieldDescriptorProto
    fdp = descriptor_pb2.FileDescriptorProto(name="dtf_tf_schema.proto", package="tfs", syntax="proto3")

    def msg(name, *fields):
        m = fdp.message_type.add(name=name)
        for fname, num, typ, label, tname in fields:
            f = m.field.add(name=fname, number=num, type=typ, label=label)
            if tname:
                f.type_name = ".tfs." + tname
        return m

    O, R = F.LABEL_OPTIONAL, F.LABEL_REPEATED
    S, B, I32, I64, FL, BO, M, E, D = (F.TYPE_STRING, F.TYPE_BYTES, F.TYPE_INT32, F.TYPE_INT64, F.TYPE_FLOAT,
                                       F.TYPE_BOOL, F.TYPE_MESSAGE, F.TYPE_ENUM, F.TYPE_DOUBLE)
    enum = fdp.enum_type.add(name="DataType")
    for nm, v in [("DT_INVALID", 0), ("DT_FLOAT", 1), ("DT_DOUBLE", 2), ("DT_INT32", 3), ("DT_UINT8", 4),
                  ("DT_STRING", 7), ("DT_INT64", 9), ("DT_BOOL", 10), ("DT_BFLOAT16", 14), ("DT_HALF", 19),
                  ("DT_FLOAT_REF", 101), ("DT_INT32_REF", 103)]:
        enum.value.add(name=nm, number=v)
    msg("Dim", ("size", 1, I64, O, None), ("name", 2, S, O, None))
    msg("TensorShapeProto", ("dim", 2, M, R, "Dim"), ("unknown_rank", 3, BO, O, None))
    msg("TensorProto", ("dtype", 1, E, O, "DataType"), ("tensor_shape", 2, M, O, "TensorShapeProto"),
        ("version_number", 3, I32, O, None), ("tensor_content", 4, B, O, None), ("float_val", 5, FL, R, None),
        ("int_val", 7, I32, R, None), ("string_val", 8, B, R, None))
    msg("ListValue", ("s", 2, B, R, None), ("i", 3, I64, R, None), ("f", 4, FL, R, None), ("b", 5, BO, R, None),
        ("type", 6, E, R, "DataType"), ("shape", 7, M, R, "TensorShapeProto"))
    msg("AttrValue", ("list", 1, M, O, "ListValue"), ("s", 2, B, O, None), ("i", 3, I64, O, None),
        ("f", 4, FL, O, None), ("b", 5, BO, O, None), ("type", 6, E, O, "DataType"),
        ("shape", 7, M, O, "TensorShapeProto"), ("tensor", 8, M, O, "TensorProto"))
    nd = msg("NodeDef", ("name", 1, S, O, None), ("op", 2, S, O, None), ("input", 3, S, R, None),
             ("device", 4, S, O, None))
    entry = nd.nested_type.add(name="AttrEntry")
    entry.field.add(name="key", number=1, type=S, label=O)
    entry.field.add(name="value", number=2, type=M, label=O, type_name=".tfs.AttrValue")
    entry.options.map_entry = True
    nd.field.add(name="attr", number=5, type=M, label=R, type_name=".tfs.NodeDef.AttrEntry")
    msg("VersionDef", ("producer", 1, I32, O, None), ("min_consumer", 2, I32, O, None))
    msg("GraphDef", ("node", 1, M, R, "NodeDef"), ("versions", 4, M, O, "VersionDef"))
    msg("SaverDef", ("filename_tensor_name", 1, S, O, None), ("save_tensor_name", 2, S, O, None),
        ("restore_op_name", 3, S, O, None), ("max_to_keep", 4, I32, O, None), ("sharded", 5, BO, O, None),
        ("keep_checkpoint_every_n_hours", 6, FL, O, None), ("version", 7, I32, O, None))
    msg("MetaInfoDef", ("meta_graph_version", 1, S, O, None), ("tags", 4, S, R, None),
        ("tensorflow_version", 5, S, O, None))
    msg("BytesList", ("value", 1, B, R, None))
    msg("NodeList", ("value", 1, S, R, None))
    msg("CollectionDef", ("node_list", 1, M, O, "NodeList"), ("bytes_list", 2, M, O, "BytesList"))
    msg("VariableDef", ("variable_name", 1, S, O, None), ("initializer_name", 2, S, O, None),
        ("snapshot_name", 3, S, O, None), ("initial_value_name", 6, S, O, None), ("trainable", 7, BO, O, None))
    msg("TensorInfo", ("name", 1, S, O, None), ("dtype", 2, E, O, "DataType"),
        ("tensor_shape", 3, M, O, "TensorShapeProto"))
    sd = msg("SignatureDef", ("method_name", 3, S, O, None))
    for fname, num in (("inputs", 1), ("outputs", 2)):
        e = sd.nested_type.add(name=fname.capitalize() + "Entry")
        e.field.add(name="key", number=1, type=S, label=O)
        e.field.add(name="value", number=2, type=M, label=O, type_name=".tfs.TensorInfo")
        e.options.map_entry = True
        sd.field.add(name=fname, number=num, type=M, label=R, type_name=f".tfs.SignatureDef.{e.name}")
    mg = msg("MetaGraphDef", ("meta_info_def", 1, M, O, "MetaInfoDef"), ("graph_def", 2, M, O, "GraphDef"),
             ("saver_def", 3, M, O, "SaverDef"))
    for fname, num, vt in (("collection_def", 4, "CollectionDef"), ("signature_def", 5, "SignatureDef")):
        e = mg.nested_type.add(name="".join(p.capitalize() for p in fname.split("_")) + "Entry")
        e.field.add(name="key", number=1, type=S, label=O)
        e.field.add(name="value", number=2, type=M, label=O, type_name=f".tfs.{vt}")
        e.options.map_entry = True
        mg.field.add(name=fname, number=num, type=M, label=R, type_name=f".tfs.MetaGraphDef.{e.name}")
    msg("SavedModel", ("saved_model_schema_version", 1, I64, O, None), ("meta_graphs", 2, M, R, "MetaGraphDef"))
    msg("Event", ("wall_time", 1, D, O, None), ("step", 2, I64, O, None), ("file_version", 3, S, O, None),
        ("graph_def", 4, B, O, None))
    pool = descriptor_pool.DescriptorPool()
    pool.Add(fdp)
    return {n: message_factory.GetMessageClass(pool.FindMessageTypeByName("tfs." + n))
            for n in ("GraphDef", "MetaGraphDef", "SavedModel", "VariableDef", "Event", "TensorProto")}


@pytest.fixture(scope="module")
def tf():
    return _tf_schema()


def _nodes(graph):
    return {n.name: n for n in graph.node}


def _check_graph(graph):
    """Every input names an existing node (control inputs '^node', outputs 'node:i'), and VersionDef is set."""
    nodes = _nodes(graph)
    for n in graph.node:
        for i in n.input:
            base = i.lstrip("^").split(":")[0]
            assert base in nodes, f"{n.name} reads missing {i}"
    assert graph.versions.producer >= 21
    return nodes


def test_linear_saved_model_is_a_tf_metagraph(tmp_path, tf):
    from distributed_tensorflow_amd import saved_model
    from distributed_tensorflow_amd.models.linear import LinearRegression
    m = LinearRegression()
    m.weight.assign(torch.tensor(2.0))
    m.bias.assign(torch.tensor(10.0))
    d = saved_model.save(m, str(tmp_path / "1"))
    sm = tf["SavedModel"]()
    sm.ParseFromString(open(os.path.join(d, "saved_model.pb"), "rb").read())
    assert sm.saved_model_schema_version == 1 and len(sm.meta_graphs) == 1
    mg = sm.meta_graphs[0]
    assert list(mg.meta_info_def.tags) == ["serve"]
    nodes = _check_graph(mg.graph_def)
    ops = {n.name: n.op for n in mg.graph_def.node}
    assert ops["keys"] == ops["features"] == "Placeholder"
    assert ops["weight"] == ops["bias"] == "VariableV2"
    assert ops["mul"] == "Mul" and ops["prediction"] == "Add" and ops["keys_identity"] == "Identity"
    assert list(nodes["prediction"].input) == ["mul", "bias/read"]
    assert list(nodes["mul"].input) == ["features", "weight/read"]
    assert nodes["keys"].attr["dtype"].type == 3 and nodes["features"].attr["dtype"].type == 1
    assert [d.size for d in nodes["keys"].attr["shape"].shape.dim] == [-1, 1]
    # the SignatureDef binds the reference's keys to real graph tensors (reference trainer/task.py:164-173)
    sig = mg.signature_def["serving_default"]
    assert sig.method_name == "tensorflow/serving/predict"
    assert sig.inputs["keys"].name == "keys:0" and sig.inputs["features"].name == "features:0"
    assert sig.outputs["keys"].name == "keys_identity:0" and sig.outputs["prediction"].name == "prediction:0"
    for ti in list(sig.inputs.values()) + list(sig.outputs.values()):
        assert ti.name.split(":")[0] in nodes
    # SaverDef (V2) names tensors / ops of the saver subgraph, which saves exactly the variables
    sd = mg.saver_def
    assert sd.version == 2 and sd.restore_op_name in nodes
    assert sd.filename_tensor_name.split(":")[0] in nodes and sd.save_tensor_name.split(":")[0] in nodes
    save = nodes["save/SaveV2"]
    tn = tf["TensorProto"]()
    tn.CopyFrom(nodes["save/SaveV2/tensor_names"].attr["value"].tensor)
    assert sorted(s.decode() for s in tn.string_val) == ["bias", "weight"]
    assert list(save.attr["dtypes"].list.type) == [1, 1]
    assert {i.lstrip("^") for i in nodes["save/restore_all"].input} == {"save/Assign", "save/Assign_1"}
    # variables collection: VariableDefs with TF naming
    vd = tf["VariableDef"]()
    vals = mg.collection_def["variables"].bytes_list.value
    names = set()
    for raw in vals:
        vd.ParseFromString(raw)
        names.add(vd.variable_name)
        assert vd.initializer_name.endswith("/Assign") and vd.snapshot_name.endswith("/read:0")
    assert names == {"weight:0", "bias:0"}
    # the variable initial values carry the exported numbers
    init = nodes["weight/initial_value"].attr["value"].tensor
    assert np.frombuffer(init.tensor_content, dtype=np.float32)[0] == 2.0
    # and the model still round-trips through this framework's loader
    loaded = saved_model.load(d)
    out = loaded.signatures["serving_default"](keys=[[11.0], [2.0]], features=[[1], [2]])
    assert out["prediction"].flatten().tolist() == [12.0, 14.0]


@pytest.mark.parametrize("opt", ["sgd", "adam", "adagrad", "adadelta", "ftrl", "rmsprop"])
def test_training_meta_graph_has_optimizer_ops_and_slots(tf, opt):
    from distributed_tensorflow_amd.keras import optimizers as O
    from distributed_tensorflow_amd.models.linear import LinearRegression
    m = LinearRegression()
    o = O.get(opt, 0.01, tf1=True)
    mg = tf["MetaGraphDef"]()
    mg.ParseFromString(GD.training_meta_graph(m, optimizer=o))
    nodes = _check_graph(mg.graph_def)
    op = LinearRegression._TF_APPLY[o.kind][0]
    applies = [n for n in mg.graph_def.node if n.op == op]
    assert len(applies) == 2 and {a.input[0] for a in applies} == {"weight", "bias"}
    for _, slots, _ in [LinearRegression._TF_APPLY[o.kind]]:
        for v in ("weight", "bias"):
            for sn in slots:
                assert nodes[f"{v}/{sn}"].op == "VariableV2"  # slot checkpoint keys of SURVEY §2.4.a
    assert nodes["global_step"].attr["dtype"].type == 3
    assert mg.collection_def["train_op"].node_list.value[0] in nodes
    assert nodes["loss"].op == "Sum" and nodes["Square"].op == "Square"
    trainable = mg.collection_def["trainable_variables"].bytes_list.value
    assert len(trainable) == 2


def test_cli_writes_graph_event_and_checkpoint_meta(tmp_path, tf):
    """The distributed runbook's artifacts: event file whose graph record is a GraphDef, model.ckpt-N.meta."""
    import subprocess
    import sys
    from distributed_tensorflow_amd.summary import read_event_records
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, PYTHONPATH=root, HIP_VISIBLE_DEVICES="", CUDA_VISIBLE_DEVICES="")
    r = subprocess.run([sys.executable, "-m", "distributed_tensorflow_amd.cli.train", "--max_epochs=2", "--seed=0"],
                       cwd=tmp_path, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout + r.stderr
    ev_files = glob.glob(str(tmp_path / "tensorboard" / "events.out.tfevents.*"))
    assert ev_files
    events = []
    for raw in read_event_records(ev_files[0]):
        e = tf["Event"]()
        e.ParseFromString(raw)
        events.append(e)
    graphs = [e for e in events if e.graph_def]
    assert graphs and events[0].file_version.startswith("brain.Event:")
    g = tf["GraphDef"]()
    g.ParseFromString(graphs[0].graph_def)
    nodes = _check_graph(g)
    assert nodes["weight"].op == "VariableV2" and nodes["GradientDescent"].op == "NoOp"


def test_supervised_checkpoint_writes_meta(tmp_path, tf):
    from distributed_tensorflow_amd.models.linear import LinearRegression
    from distributed_tensorflow_amd.train.checkpoint import Saver, latest_checkpoint
    m = LinearRegression()
    s = Saver({"weight": m.weight, "bias": m.bias}, meta_graph_def=lambda: GD.training_meta_graph(m))
    prefix = s.save(save_path=str(tmp_path / "model.ckpt"), global_step=7)
    assert latest_checkpoint(str(tmp_path)) == prefix and prefix.endswith("model.ckpt-7")
    mg = tf["MetaGraphDef"]()
    mg.ParseFromString(open(prefix + ".meta", "rb").read())
    assert mg.saver_def.version == 2
    _check_graph(mg.graph_def)
