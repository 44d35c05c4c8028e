"""Distributed training on CPU: MultiWorkerMirroredStrategy over 2 processes (shared-memory and gloo
all-reduce), the in-process MirroredStrategy(CPU:0, CPU:1) plumbing config of BASELINE.json, the
gradient bucketer, and ParameterServerStrategy driven through Keras Model.fit."""
import json
import multiprocessing as mp
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _train_mlp(strategy, x, y, epochs=2, batch=64, seed=0):
    from distributed_tensorflow_amd.keras import initializers, losses, optimizers
    from distributed_tensorflow_amd.models.mlp import MnistMLP
    initializers.set_seed(seed)
    with strategy.scope():
        m = MnistMLP(hidden=32)
        m.compile(optimizers.SGD(0.1, momentum=0.9), losses.SparseCategoricalCrossentropy(from_logits=True),
                  metrics=["accuracy"])
    h = m.fit(x, y, batch_size=batch, epochs=epochs, shuffle=False, verbose=0)
    return m, h


def _mwms_worker(rank, world, port, mode, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port), DTF_CPU_ALLREDUCE=mode.split("_")[0], HIP_VISIBLE_DEVICES="",
                      CUDA_VISIBLE_DEVICES="", DTF_ALLREDUCE_DTYPE="bf16" if mode.endswith("bf16") else "f32",
                      DTF_ZERO="1" if "zero" in mode else "0",
                      DTF_BUCKET_MB="0.0001" if ("zero" in mode or "ovl" in mode) else "32",
                      DTF_OVERLAP_UPDATE="force" if "ovl" in mode else "0")
    try:
        from distributed_tensorflow_amd import parallel
        from distributed_tensorflow_amd.models.mlp import synthetic_mnist
        n, batch = (576, 96) if world == 3 else (512, 64)
        x, y = synthetic_mnist(n)
        s = parallel.MultiWorkerMirroredStrategy()
        # every rank starts from its own random init: rank 0's must be broadcast before the first step
        m, h = _train_mlp(s, torch.as_tensor(x), torch.as_tensor(y), seed=rank, batch=batch)
        from distributed_tensorflow_amd.parallel.collective import ShardedGradientBucketer
        assert ("zero" in mode) == any(isinstance(b, ShardedGradientBucketer) for b in s._bucketers.values())
        s.sync_optimizer_state(m.optimizer)  # ZeRO-1: make every replica's slots whole (no-op otherwise)
        slots = [m.optimizer.get_slot(v, "Momentum").detach().numpy().copy() for v in m.trainable_variables]
        q.put((rank, [w.detach().numpy().copy() for w in m.weights] + slots, h.history["loss"]))
        import torch.distributed as dist
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # surface the failure to the parent
        import traceback
        q.put((rank, None, traceback.format_exc()))


@pytest.mark.parametrize("mode,world", [("shm", 2), ("gloo", 2), ("gloo_bf16", 2), ("gloo_zero", 2),
                                        ("gloo_zero", 3), ("gloo_zero_bf16", 2), ("gloo_ovl", 2), ("gloo_ovl_bf16", 2)])
def test_multi_worker_mirrored_matches_single_process(mode, world):
    """gloo_bf16: the gradient buckets travel as bf16 (half the all-reduce bytes) and are accumulated back into
    the f32 arena; the replicas still agree exactly and track f32 training within bf16 rounding.
    gloo_zero: ZeRO-1 (reduce-scatter, 1/N optimizer update per replica, all-gather of the masters; tiny
    buckets so every variable boundary case is hit; world 3 exercises the padded, non-divisible chunks) —
    weights AND the gathered momentum slots equal single-process training.
    gloo_ovl: the optimizer update runs bucket by bucket inside backward, right after each bucket's all-reduce
    (tiny buckets: many partial updates per step) — same result as the update after backward."""
    from distributed_tensorflow_amd import parallel
    from distributed_tensorflow_amd.models.mlp import synthetic_mnist
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_mwms_worker, args=(r, world, port, mode, q)) for r in range(world)]
    [p.start() for p in ps]
    res = sorted([q.get(timeout=240) for _ in range(world)], key=lambda t: t[0])
    [p.join(60) for p in ps]
    for r in res:
        assert r[1] is not None, r[2]
    # all replicas hold identical weights (and slots)
    for other in res[1:]:
        for a, b in zip(res[0][1], other[1]):
            np.testing.assert_allclose(a, b, rtol=0, atol=0)
    # and equal single-process training on the same global batches
    n, batch = (576, 96) if world == 3 else (512, 64)
    x, y = synthetic_mnist(n)
    m, h = _train_mlp(parallel.OneDeviceStrategy("cpu"), torch.as_tensor(x), torch.as_tensor(y), batch=batch)
    tol = dict(rtol=2e-2, atol=2e-3) if mode.endswith("bf16") else dict(rtol=1e-4, atol=1e-5)
    ref = [w.detach().numpy() for w in m.weights] + [m.optimizer.get_slot(v, "Momentum").detach().numpy()
                                                     for v in m.trainable_variables]
    for a, w in zip(res[0][1], ref):
        np.testing.assert_allclose(a, w, **tol)
    assert res[0][2][-1] < res[0][2][0]


def test_mirrored_cpu0_cpu1_plumbing_config():
    """BASELINE.json config 1: MNIST 2-layer MLP, MirroredStrategy on CPU:0,CPU:1."""
    from distributed_tensorflow_amd import parallel
    from distributed_tensorflow_amd.models.mlp import synthetic_mnist
    x, y = synthetic_mnist(512)
    X, Y = torch.as_tensor(x), torch.as_tensor(y)
    s = parallel.MirroredStrategy(["CPU:0", "CPU:1"])
    assert s.num_replicas_in_sync == 2
    m2, h2 = _train_mlp(s, X, Y)
    m1, h1 = _train_mlp(parallel.OneDeviceStrategy("cpu"), X, Y)
    for a, b in zip(m2.weights, m1.weights):
        np.testing.assert_allclose(a.detach().numpy(), b.detach().numpy(), rtol=1e-4, atol=1e-5)
    assert h2.history["accuracy"][-1] > 0.5


def test_gradient_buckets_cover_arena_in_reverse_order():
    from distributed_tensorflow_amd import Variable
    from distributed_tensorflow_amd.parallel.collective import GradientBucketer
    from distributed_tensorflow_amd.variables import ParamArena
    vs = [Variable(torch.randn(n), name=f"v{i}") for i, n in enumerate([1000, 3, 70000, 12, 500000, 7])]
    a = ParamArena(vs)
    b = GradientBucketer(a, bucket_mb=0.5)
    cover = sorted(b.buckets)
    assert cover[0][0] == 0 and cover[-1][1] == a.numel
    for (l0, h0), (l1, h1) in zip(cover, cover[1:]):
        assert h0 == l1
    # bucket 0 holds the LAST variables (produced first by backward)
    assert b.var_bucket[-1] == 0 and b.var_bucket[0] == len(b.buckets) - 1
    assert sorted(b.var_bucket, reverse=True) == b.var_bucket


PS_SCRIPT = r"""
import os, sys, json, torch
from distributed_tensorflow_amd.parallel import TFConfigClusterResolver, ParameterServerStrategy, run_parameter_server
from distributed_tensorflow_amd.keras import losses, optimizers, initializers
from distributed_tensorflow_amd.models.mlp import MnistMLP, synthetic_mnist
r = TFConfigClusterResolver()
if r.is_ps:
    sys.exit(run_parameter_server(r, device="cpu"))
s = ParameterServerStrategy(r, variable_partitioner="balanced", device="cpu")
initializers.set_seed(0)
x, y = synthetic_mnist(512, seed=1 + s.worker_index)
with s.scope():
    m = MnistMLP(hidden=32)
    m.compile(optimizers.Adam(0.01), losses.SparseCategoricalCrossentropy(from_logits=True), metrics=["accuracy"])
h = m.fit(torch.as_tensor(x), torch.as_tensor(y), batch_size=32, epochs=3, verbose=0)
s.pull()
acc = m.evaluate(torch.as_tensor(x), torch.as_tensor(y), verbose=0, return_dict=True)["accuracy"]
print(json.dumps({"task": r.task_type, "acc": acc, "gs": s.global_step(), "loss": h.history["loss"]}), flush=True)
s.shutdown()
"""


@pytest.mark.slow
def test_parameter_server_strategy_keras_fit(tmp_path):
    script = tmp_path / "ps_fit.py"
    script.write_text(PS_SCRIPT)
    env = dict(os.environ, PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable, "-m", "distributed_tensorflow_amd.cli.launch", "--ps", "2", "--workers", "2",
                        "--chief", "1", "--chief_job", "chief", "--timeout", "240", "--", sys.executable,
                        str(script)], env=env, capture_output=True, text=True, timeout=300, cwd=tmp_path)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out
    res = [json.loads(l.split("] ", 1)[1]) for l in out.splitlines() if '"acc"' in l]
    assert len(res) == 3
    for d in res:
        assert d["acc"] > 0.8, out
        assert d["loss"][-1] < d["loss"][0]
    assert max(d["gs"] for d in res) >= 3 * 16  # async global_step counts every worker's steps


@pytest.mark.slow
@pytest.mark.parametrize("transport", ["", "tcp"])
def test_ps_runbook_negotiated_transport(tmp_path, transport):
    """The PS runbook with the data plane the chief negotiates for the whole cluster (unset: every task on one host
    -> 'shm', direct copies into the PS's memory + the native mailbox) or forced to 'tcp' through the chief's
    environment: 2 PS + 1 worker + master, ASSIGN/PUSH/pull per shard, DONE-driven PS exit, export, checkpoint."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ)
    env.pop("DTF_PS_TRANSPORT", None)
    if transport:
        env["DTF_PS_TRANSPORT"] = transport
    env["PYTHONPATH"] = root + (os.pathsep + env["PYTHONPATH"] if env.get("PYTHONPATH") else "")
    cmd = [sys.executable, "-m", "distributed_tensorflow_amd.cli.launch", "--ps", "2", "--workers", "1", "--chief",
           "1", "--timeout", "240", "--", sys.executable, "-m", "distributed_tensorflow_amd.cli.train", "--seed=0",
           "--max_epochs=4", "--optimizer=adam", "--learning_rate=0.1"]
    r = subprocess.run(cmd, cwd=tmp_path, env=env, capture_output=True, text=True, timeout=300)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert out.count("PS exits after all workers done") == 2
    assert "Exported SavedModel" in out
    assert f"PS data plane: {transport or 'shm'}" in out
    from distributed_tensorflow_amd.train import checkpoint as C
    ck = C.latest_checkpoint(str(tmp_path / "checkpoint"))
    names = dict(C.list_variables(ck))
    assert {"weight", "bias", "global_step"} <= set(names)
    w = float(C.load_variable(ck, "weight"))
    assert 1.0 < w < 3.0, w


@pytest.mark.slow
@pytest.mark.parametrize("staleness", ["0", "1"])
def test_ps_shm_two_ps_six_trainers(tmp_path, staleness):
    """BASELINE config 4's topology (2 PS + 6 trainers) on the CPU through ONE serve loop per PS: 6 trainers
    (master + 5 workers) push/pull concurrently through the shared-memory mailbox; every update is applied
    (global_step counts all of them) and the model converges (async SGD, reference trainer/task.py:232-236).
    staleness 1: pushes return once the PS consumed the inbox (OP_PUSH_ASYNC), the trainer only waits for that
    acknowledgement before refilling its inbox on the next push — still every push applied exactly once."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, OMP_NUM_THREADS="1", DTF_PS_STALENESS=staleness)
    env.pop("DTF_PS_TRANSPORT", None)
    env["PYTHONPATH"] = root + (os.pathsep + env["PYTHONPATH"] if env.get("PYTHONPATH") else "")
    cmd = [sys.executable, "-m", "distributed_tensorflow_amd.cli.launch", "--ps", "2", "--workers", "5", "--chief",
           "1", "--timeout", "280", "--", sys.executable, "-m", "distributed_tensorflow_amd.cli.train", "--seed=0",
           "--max_epochs=2", "--optimizer=sgd", "--learning_rate=0.01"]
    r = subprocess.run(cmd, cwd=tmp_path, env=env, capture_output=True, text=True, timeout=320)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert out.count("PS exits after all workers done") == 2
    assert out.count("PS data plane: shm") >= 8
    from distributed_tensorflow_amd.train import checkpoint as C
    ck = C.latest_checkpoint(str(tmp_path / "checkpoint"))
    gs = int(C.load_variable(ck, "global_step"))
    assert 2 * 100 <= gs <= 6 * 2 * 100, gs  # the chief saved while the other trainers were still stepping
    import re
    applied = [int(m) for m in re.findall(r"PS applied (\d+) updates", out)]
    assert applied == [6 * 2 * 100] * 2, applied  # every trainer's every push reached both shards
    w, b = float(C.load_variable(ck, "weight")), float(C.load_variable(ck, "bias"))
    assert 1.5 < w < 2.5 and 9.5 < b < 10.5, (w, b)


def test_mirrored_over_gpu_list_runs_one_process_per_device(tmp_path):
    """MirroredStrategy(["GPU:0", "GPU:1"]) re-runs the program once per listed device (the parent exits with the
    children's status); each child is one rank of the multi-process strategy and reduces with the others (gloo here:
    no GPU in this container; tests/test_dp_gpu.py trains through it on a GPU). Mixed GPU/host lists are rejected."""
    import subprocess
    import sys
    import pytest
    from distributed_tensorflow_amd import parallel
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    script = tmp_path / "m.py"
    script.write_text(
        "import sys, os\n"
        f"sys.path.insert(0, {root!r})\n"
        "import torch\n"
        "from distributed_tensorflow_amd import parallel\n"
        "s = parallel.MirroredStrategy(['GPU:0', 'GPU:1'])\n"
        "t = s.reduce('sum', torch.tensor(float(s.worker_index + 1)))\n"
        f"open(os.path.join({str(tmp_path)!r}, 'r%d' % s.worker_index), 'w').write("
        "'%d %d %g' % (s.worker_index, s.num_replicas_in_sync, float(t)))\n")
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    r = subprocess.run([sys.executable, str(script)], env=env, timeout=240)
    assert r.returncode == 0
    for k in range(2):
        assert (tmp_path / f"r{k}").read_text() == f"{k} 2 3"
    with pytest.raises(ValueError, match="mixing"):
        parallel.MirroredStrategy(["GPU:0", "GPU:1", "CPU:0"])


def test_overlapped_bucket_update_matches_single_update(monkeypatch):
    """One replica: the per-bucket optimizer update inside backward (collective-free GradientBucketer, forced on
    for a CPU arena) trains exactly like one fused update after backward — SGD+momentum and Adam, tiny buckets."""
    from distributed_tensorflow_amd import parallel
    from distributed_tensorflow_amd.keras import initializers, losses, optimizers
    from distributed_tensorflow_amd.models.mlp import MnistMLP, synthetic_mnist
    from distributed_tensorflow_amd.parallel import collective, strategy as S
    x, y = synthetic_mnist(256)
    X, Y = torch.as_tensor(x), torch.as_tensor(y)

    def run(mode, opt):
        monkeypatch.setattr(S, "_OVERLAP_UPDATE", mode)
        monkeypatch.setattr(collective, "_DEFAULT_BUCKET_MB", 0.0001)
        initializers.set_seed(0)
        s = parallel.OneDeviceStrategy("cpu")
        with s.scope():
            m = MnistMLP(hidden=32)
            m.compile(opt(), losses.SparseCategoricalCrossentropy(from_logits=True))
        m.fit(X, Y, batch_size=64, epochs=2, shuffle=False, verbose=0)
        nb = len(s._bucketers[id(m._arena)].buckets) if s._bucketers else 0
        return [w.detach().numpy().copy() for w in m.weights], int(m.optimizer.iterations.item()), nb

    for opt in (lambda: optimizers.SGD(0.1, momentum=0.9), lambda: optimizers.Adam(1e-2)):
        a, ia, nb = run("force", opt)
        b, ib, _ = run("0", opt)
        assert nb > 2 and ia == ib == 8
        for u, v in zip(a, b):
            np.testing.assert_allclose(u, v, rtol=1e-6, atol=1e-7)


def test_launcher_gpu_ordinals_keep_callers_visible_set():
    """cli.launch --gpus: every chief/worker task gets DTF_DEVICE_ORDINAL = its entry of --gpus, an index INTO the
    caller's visible devices, and the caller's HIP_VISIBLE_DEVICES passes through unchanged (popping it
    turned --gpus indices into physical ids outside the allowed set)."""
    import io
    import sys
    from distributed_tensorflow_amd.cli.launch import launch
    code = ("import os, json; print(json.dumps({'role': os.environ['DTF_ROLE'], "
            "'ord': os.environ.get('DTF_DEVICE_ORDINAL'), 'vis': os.environ.get('HIP_VISIBLE_DEVICES')}))")
    buf = io.StringIO()
    rc, _ = launch([sys.executable, "-c", code], num_ps=1, num_workers=1, num_chief=1, gpus="1,0",
                   env={"HIP_VISIBLE_DEVICES": "3,5"}, timeout=60, log=buf)
    assert rc == 0, buf.getvalue()
    import json
    got = {d["role"]: d for d in (json.loads(l.split("] ", 1)[1]) for l in buf.getvalue().splitlines() if "{" in l)}
    assert got["master0"]["ord"] == "1" and got["worker0"]["ord"] == "0", got
    assert got["master0"]["vis"] == "3,5" and got["worker0"]["vis"] == "3,5", got
    assert got["ps0"]["ord"] is None and got["ps0"]["vis"] == "", got  # PS on CPU unless --ps_gpus


def test_agree_exchanges_only_every_nth_call(monkeypatch):
    """ZeRO-1 + a wall-clock checkpoint trigger: rank 0's decision is broadcast only every `every`-th batch, never
    per batch."""
    from distributed_tensorflow_amd.parallel import strategy as S
    s = S.MultiWorkerMirroredStrategy.__new__(S.MultiWorkerMirroredStrategy)
    s._world, s.shard_optimizer, s._device = 2, True, torch.device("cpu")
    calls = []
    monkeypatch.setattr(S.dist, "broadcast", lambda t, src=0: calls.append(int(t.item())))
    out = [s.agree(True, every=4) for _ in range(8)]
    assert out == [False, False, False, True] * 2 and len(calls) == 2


def test_native_rccl_binding_and_selection():
    """The C++ RCCL communicator binds librccl at run time (PyTorch's copy when loaded) on any host; the bucketer's
    communicator choice follows CommunicationImplementation (NCCL -> ours, RING -> torch's process group)."""
    from distributed_tensorflow_amd.parallel import rccl, CommunicationOptions, CommunicationImplementation
    ok, where = rccl.available()
    assert ok, where
    assert rccl.version() >= 22000
    assert rccl.wanted(CommunicationImplementation.NCCL) and not rccl.wanted(CommunicationImplementation.RING)
    assert rccl.wanted("rccl") and not rccl.wanted("torch")
    co = CommunicationOptions(implementation="nccl")
    assert co.implementation is CommunicationImplementation.NCCL
    assert CommunicationOptions().implementation is CommunicationImplementation.AUTO
