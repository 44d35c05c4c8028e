"""Reference-behaviour tests (CPU): flags, TF_CONFIG, TF1 optimizer oracle,
standalone linear training, the 3-process PS cluster with auto-stop, export + REST serving."""
import json
import os
import subprocess
import sys
import threading
import urllib.request

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env():
    e = dict(os.environ)
    e["PYTHONPATH"] = ROOT + (os.pathsep + e["PYTHONPATH"] if e.get("PYTHONPATH") else "")
    e["HIP_VISIBLE_DEVICES"] = ""
    e["CUDA_VISIBLE_DEVICES"] = ""
    return e


# ------------------------------------------------------------------ flags / cluster
def test_flags_defaults_and_parse():
    from distributed_tensorflow_amd.utils.flags import _FlagValues
    f = _FlagValues()
    f._define("max_epochs", 10, "", int)
    f._define("optimizer", "sgd", "", str)
    f._define("learning_rate", 0.01, "", float)
    f._define("flag", False, "", bool)
    rest = f(["--max_epochs=3", "--optimizer", "adam", "--unknown=1", "--flag", "pos"])
    assert f.max_epochs == 3 and f.optimizer == "adam" and f.learning_rate == 0.01 and f.flag is True
    assert "--unknown=1" in rest and "pos" in rest


def test_cli_flag_defaults_match_reference():
    from distributed_tensorflow_amd.cli import train  # noqa: F401  (defines the flags)
    from distributed_tensorflow_amd.utils.flags import FLAGS
    FLAGS.reset()
    FLAGS([])
    # reference trainer/task.py:17-31
    assert FLAGS.max_epochs == 10
    assert FLAGS.checkpoint_path == "./checkpoint/"
    assert FLAGS.output_path == "./tensorboard/"
    assert FLAGS.checkpoint_period == 1
    assert FLAGS.model_path == "./model/"
    assert FLAGS.learning_rate == 0.01
    assert FLAGS.optimizer == "sgd"
    assert FLAGS.saved_model_path == "./saved_model/"
    assert FLAGS.model_version == 1


def test_tf_config_resolver():
    from distributed_tensorflow_amd.parallel import TFConfigClusterResolver
    cfg = {"cluster": {"ps": ["127.0.0.1:3001"], "worker": ["127.0.0.1:3002"], "master": ["127.0.0.1:3003"]},
           "task": {"index": 0, "type": "master"}}
    r = TFConfigClusterResolver(json.dumps(cfg))
    assert r.is_chief and not r.is_ps and not r.standalone
    assert r.cluster.num_tasks("ps") == 1
    assert r.trainer_tasks() == [("master", 0), ("worker", 0)]
    w = TFConfigClusterResolver({**cfg, "task": {"type": "worker", "index": 0}})
    assert not w.is_chief and w.trainer_rank() == 1
    c = TFConfigClusterResolver({"cluster": {"chief": ["a:1"], "worker": ["b:2"]}, "task": {"type": "chief"}})
    assert c.is_chief
    nochief = TFConfigClusterResolver({"cluster": {"worker": ["a:1", "b:2"]}, "task": {"type": "worker", "index": 0}})
    assert nochief.is_chief
    assert TFConfigClusterResolver("").standalone
    with pytest.raises(ValueError):
        TFConfigClusterResolver({"cluster": {"worker": ["a:1"]}, "task": {"type": "bogus", "index": 0}})


# ------------------------------------------------------------------ optimizer oracle
ORACLE = {  # (optimizer, epochs) -> (w, b) with RandomState(0) data, batch 1, lr 0.01
    ("sgd", 10): (2.031, 10.021),
    ("sgd", 20): (2.039, 10.018),
    ("adam", 10): (0.974, 7.482),
    ("rmsprop", 10): (2.244, 9.666),
    ("adagrad", 10): (0.008, 0.623),
    ("ftrl", 10): (0.008, 0.623),
    ("adadelta", 10): (0.0007, 0.007),
}


@pytest.mark.parametrize("key", sorted(ORACLE))
def test_linear_regression_matches_tf1_oracle(key):
    from distributed_tensorflow_amd.data import reference_linear_data
    from distributed_tensorflow_amd.keras import optimizers
    from distributed_tensorflow_amd.models.linear import LinearRegression
    name, epochs = key
    x, y = reference_linear_data(0)
    m = LinearRegression()
    opt = optimizers.get(name, 0.01, tf1=True)
    arena = opt.arena_for(m.trainable_variables)
    loss_fn = LinearRegression.reference_loss()
    X = torch.as_tensor(x).reshape(-1, 1, 1)
    Y = torch.as_tensor(y).reshape(-1, 1, 1)
    for _ in range(epochs):
        for j in range(100):
            loss_fn(Y[j], m(X[j])).backward()
            opt.apply_arena(arena)
    w, b = ORACLE[key]
    assert abs(float(m.weight) - w) < max(2e-3, 2e-3 * abs(w)), (float(m.weight), w)
    assert abs(float(m.bias) - b) < max(2e-3, 2e-3 * abs(b)), (float(m.bias), b)


def test_unknown_optimizer_exits_1(tmp_path):
    r = subprocess.run([sys.executable, "-m", "distributed_tensorflow_amd.cli.train", "--optimizer=bogus"],
                       cwd=tmp_path, env=_env(), capture_output=True, text=True, timeout=120)
    assert r.returncode == 1
    assert "Unknow optimizer: bogus" in r.stdout


def test_standalone_cli_end_to_end(tmp_path):
    r = subprocess.run([sys.executable, "-m", "distributed_tensorflow_amd.cli.train", "--seed=0", "--max_epochs=10",
                        "--export_standalone"], cwd=tmp_path, env=_env(), capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "Epoch: 9, loss:" in r.stdout
    line = [l for l in r.stdout.splitlines() if l.startswith("Get the model")][0]
    w = float(line.split("w: ")[1].split(",")[0])
    b = float(line.split("b: ")[1])
    assert abs(w - 2.031) < 2e-3 and abs(b - 10.021) < 2e-3
    # summaries: loss and the hptuning metric every epoch
    from distributed_tensorflow_amd import summary
    ev = [f for f in os.listdir(tmp_path / "tensorboard") if f.startswith("events.out")]
    recs = summary.read_events(str(tmp_path / "tensorboard" / ev[0]))
    tags = [set(v) for _, _, v in recs]
    assert sum("loss" in t for t in tags) == 10
    assert sum("training/hptuning/metric" in t for t in tags) == 10


@pytest.mark.slow
def test_ps_cluster_runbook_with_auto_stop(tmp_path):
    """README.md:9-27: ps + worker + master on 127.0.0.1; PS tasks exit by themselves."""
    cmd = [sys.executable, "-m", "distributed_tensorflow_amd.cli.launch", "--ps", "2", "--workers", "1", "--chief",
           "1", "--timeout", "240", "--", sys.executable, "-m", "distributed_tensorflow_amd.cli.train", "--seed=0",
           "--max_epochs=4", "--optimizer=sgd"]
    r = subprocess.run(cmd, cwd=tmp_path, env=_env(), capture_output=True, text=True, timeout=300)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out
    assert out.count("PS exits after all workers done") == 2
    assert "Exported SavedModel" in out
    ck = [f for f in os.listdir(tmp_path / "checkpoint") if f.endswith(".index")]
    assert ck, os.listdir(tmp_path / "checkpoint")
    from distributed_tensorflow_amd.train import checkpoint as C
    names = dict(C.list_variables(str(tmp_path / "checkpoint" / ck[0][:-6])))
    assert set(names) == {"weight", "bias", "global_step"}
    w = float(C.load_variable(str(tmp_path / "checkpoint" / ck[0][:-6]), "weight"))
    assert 1.5 < w < 2.5  # two async replicas on the same data converge near w=2


def test_export_and_rest_serving(tmp_path):
    from distributed_tensorflow_amd import saved_model, serving
    from distributed_tensorflow_amd.models.linear import LinearRegression
    m = LinearRegression()
    m.weight.assign(2.0)
    m.bias.assign(10.0)
    saved_model.save(m, str(tmp_path / "saved_model" / "1"))
    pb = saved_model.parse_saved_model(open(tmp_path / "saved_model" / "1" / "saved_model.pb", "rb").read())
    sig = pb["meta_graphs"][0]["signatures"]["serving_default"]
    assert pb["meta_graphs"][0]["tags"] == ["serve"]
    assert sig["method_name"] == "tensorflow/serving/predict"
    assert sig["inputs"] == {"features": ("float32", [-1, 1]), "keys": ("int32", [-1, 1])}
    assert set(sig["outputs"]) == {"keys", "prediction"}
    httpd, ms = serving.serve(str(tmp_path / "saved_model"), port=0, block=False)
    try:
        port = httpd.server_address[1]
        body = json.dumps({"keys": [[11.0], [2.0]], "features": [[1], [2]]}).encode()  # README.md:40 verbatim
        req = urllib.request.Request(f"http://127.0.0.1:{port}", data=body, headers={"Content-Type":
                                                                                        "application/json"})
        res = json.loads(urllib.request.urlopen(req, timeout=10).read())
        assert res["keys"] == [[11], [2]]
        assert np.allclose(res["prediction"], [[12.0], [14.0]])
        env = json.dumps({"model_name": "default", "data": {"keys": [[1]], "features": [[0.5]]}}).encode()
        res2 = json.loads(urllib.request.urlopen(urllib.request.Request(f"http://127.0.0.1:{port}", data=env),
                                                 timeout=10).read())
        assert np.allclose(res2["prediction"], [[11.0]])
    finally:
        httpd.shutdown()
