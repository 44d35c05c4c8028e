"""Multi-process data parallelism on the GPU path, rehearsed on ONE MI355X.

Two ranks share cuda:0 and reduce over gloo (``DTF_COLLECTIVE_BACKEND=gloo``; RCCL refuses two ranks on
one device). Everything else is the production path the 8-GPU bench takes: MultiWorkerMirroredStrategy
under torchrun-style env, initial-state broadcast, the HIP kernels with direct arena-gradient
accumulation, the bucketed all-reduce issued from post-accumulate hooks while backward runs (tiny
buckets here, so there are many of them), 1/N folded into the fused optimizer.

* GPT-2 (LayerNorm only, no batch statistics): 2 ranks x half batch must equal one process on the whole
  batch, and both replicas must hold identical weights.
* ResNet (BatchNorm statistics are per replica, as in tf.distribute): replicas must stay identical.
"""
import multiprocessing as mp

import numpy as np
import os
import socket
import traceback

import pytest
import torch

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _gpt2(seed):
    from distributed_tensorflow_amd.keras import initializers, losses, optimizers
    from distributed_tensorflow_amd.models.transformer import GPT2
    initializers.set_seed(seed)
    m = GPT2(vocab=320, ctx=128, hidden=128, layers=2, heads=2, dropout=0.0)
    # SGD, not Adam: Adam's per-element normalisation turns rounding noise in near-zero gradients into
    # full-size steps, which would hide a wrong reduction scale instead of exposing it
    m.compile(optimizer=optimizers.SGD(0.1, momentum=0.9),
              loss=losses.SparseCategoricalCrossentropy(from_logits=True))
    return m


def _resnet(seed):
    from distributed_tensorflow_amd.keras import initializers, losses, optimizers
    from distributed_tensorflow_amd.models import ResNet
    initializers.set_seed(seed)
    m = ResNet(50, num_classes=16, width=16)
    m.compile(optimizer=optimizers.SGD(0.05, momentum=0.9),
              loss=losses.SparseCategoricalCrossentropy(from_logits=True))
    return m


def _batches(kind, dev, steps=3):
    g = torch.Generator().manual_seed(5)
    out = []
    for _ in range(steps):
        if kind == "gpt2":
            ids = torch.randint(0, 320, (8, 128), generator=g)
            out.append((ids.to(dev), torch.roll(ids, -1, 1).to(dev)))
        else:
            out.append((torch.randn(8, 3, 64, 64, generator=g).to(dev), torch.randint(0, 16, (8,), generator=g).to(dev)))
    return out


def _worker(rank, world, port, kind, q, p2p="0"):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port), DTF_COLLECTIVE_BACKEND="gloo", DTF_P2P=p2p)
    try:
        import torch.distributed as dist
        from distributed_tensorflow_amd import parallel
        s = parallel.MultiWorkerMirroredStrategy(bucket_mb=0.25)
        assert s.device == torch.device("cuda", 0) and s.num_replicas_in_sync == world
        with s.scope():
            m = _gpt2(100 + rank) if kind == "gpt2" else _resnet(100 + rank)  # rank 0's init wins (broadcast)
        losses = []
        per = 8 // world
        for x, y in _batches(kind, s.device):
            sl = slice(rank * per, (rank + 1) * per)
            losses.append(float(m.train_step((x[sl], y[sl]))["loss"]))
        torch.cuda.synchronize()
        b = s._bucketers[id(m._arena)]
        # numpy, not torch CPU tensors: those travel as shared-memory fds that vanish when the worker exits
        q.put((rank, [w.detach().float().cpu().numpy() for w in m.trainable_variables], losses, len(b.buckets),
               dict(b.paths)))
        dist.barrier()
        dist.destroy_process_group()
    except Exception:
        q.put((rank, None, traceback.format_exc(), 0))


def _run_ranks(kind, world=2, p2p="0"):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, kind, q, p2p)) for r in range(world)]
    [p.start() for p in ps]
    try:
        res = sorted([q.get(timeout=100) for _ in range(world)], key=lambda t: t[0])
    finally:
        for p in ps:
            p.join(30)
            if p.is_alive():
                p.kill()
    for r in res:
        assert r[1] is not None, r[2]
    return res


def test_two_rank_gpt2_equals_single_process(cuda):
    res = _run_ranks("gpt2")
    assert res[0][3] > 3, "expected several gradient buckets"
    for a, b in zip(res[0][1], res[1][1]):
        assert (a == b).all(), "replicas diverged"
    m = _gpt2(100)
    for x, y in _batches("gpt2", cuda):
        m.train_step((x, y))
    torch.cuda.synchronize()
    for a, w in zip(res[0][1], m.trainable_variables):
        torch.testing.assert_close(torch.from_numpy(a), w.detach().float().cpu(), rtol=2e-3, atol=2e-4)


def test_two_rank_bucketer_p2p_equals_collective(cuda):
    """The gradient bucketer with the one-shot P2P all-reduce (DTF_P2P=1: small buckets on the communication stream,
    the rest on the process group, per-bucket hooks during backward) trains bitwise like the process-group-only run
    (end-to-end coverage of the bucketer integration). Two ranks share GPU 0."""
    a = _run_ranks("gpt2", p2p="1")
    b = _run_ranks("gpt2", p2p="0")
    assert a[0][4]["p2p"] > 0, a[0][4]
    assert b[0][4]["p2p"] == 0, b[0][4]
    for x, y in zip(a[0][1], b[0][1]):
        assert (x == y).all(), "P2P buckets changed the training result"
    for x, y in zip(a[0][1], a[1][1]):
        assert (x == y).all(), "replicas diverged"


def test_two_rank_resnet_replicas_stay_identical(cuda):
    res = _run_ranks("resnet")
    for a, b in zip(res[0][1], res[1][1]):
        assert (a == b).all(), "replicas diverged"
    assert all(x == x for x in res[0][2])


def _worker_rccl1(port, jit, wire, q, zero=False, impl="AUTO"):
    """One replica on the REAL RCCL backend (world size 1, DTF_FORCE_COLLECTIVE): process group, bucketed
    all-reduces from post-accumulate hooks, optionally the bf16 wire and hipGraph capture of the whole step.
    impl: CommunicationImplementation — NCCL / AUTO the framework's C++ communicator, RING torch's process group."""
    os.environ.update(RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                      DTF_FORCE_COLLECTIVE="1")
    os.environ.pop("DTF_COLLECTIVE_BACKEND", None)
    try:
        import torch.distributed as dist
        from distributed_tensorflow_amd import parallel
        s = parallel.MultiWorkerMirroredStrategy(bucket_mb=0.25,
                                                 communication_options=parallel.CommunicationOptions(
                                                     wire_dtype=wire, implementation=impl), shard_optimizer=zero)
        assert dist.get_backend() == "nccl"
        with s.scope():
            m = _gpt2(100)
        m._jit = jit
        fn = m.make_train_function(force=True)
        losses = [float(fn((x, y))["loss"]) for x, y in _batches("gpt2", s.device, steps=5)]
        torch.cuda.synchronize()
        b = s._bucketers[id(m._arena)]
        kind = type(fn).__name__ + (":captured" if getattr(fn, "captured", False) else "")
        q.put((kind, [w.detach().float().cpu().numpy() for w in m.trainable_variables], losses,
               len(b.buckets), dict(b.paths)))
        dist.destroy_process_group()
    except Exception:
        q.put((None, None, traceback.format_exc(), 0, None))


@pytest.mark.parametrize("jit,wire,zero,impl", [(False, "f32", False, "AUTO"), (True, "f32", False, "AUTO"),
                                                (False, "bf16", False, "AUTO"), (True, "bf16", False, "AUTO"),
                                                (False, "f32", True, "AUTO"), (True, "f32", True, "AUTO"),
                                                (False, "f32", True, "RING"),
                                                (False, "f32", False, "RING"), (True, "f32", False, "RING")])
def test_rccl_bucketer_world1_matches_single_process(cuda, jit, wire, zero, impl):
    """zero=True: ZeRO-1 on RCCL (reduce-scatter into the compact shard gradient, segment-wise fused AdamW, in-place
    all-gather of the masters, bf16 refresh). impl AUTO: the buckets go through the framework's own RCCL communicator
    (parallel/rccl.py) on the communication stream; RING: torch's process group. jit: the multi-rank step is captured
    as per-stream hipGraphs when the collectives are the native communicator's (the default), and stays eager on
    torch's process group."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker_rccl1, args=(_port(), jit, wire, q, zero, impl))
    p.start()
    try:
        kind, ws, losses, nb, paths = q.get(timeout=100)
    finally:
        p.join(30)
        if p.is_alive():
            p.kill()
    assert ws is not None, losses
    want = "method" if not jit else ("CapturedStep:captured" if impl == "AUTO" else "CapturedStep")
    assert nb > 3 and kind == want, kind
    native = impl == "AUTO"  # which communicator carried the buckets
    assert (paths["rccl_native"] > 0) == native and (paths["rccl"] > 0) == (not native), paths
    m = _gpt2(100)
    ref = [float(m.train_step((x, y))["loss"]) for x, y in _batches("gpt2", cuda, steps=5)]
    torch.cuda.synchronize()
    tol = dict(rtol=2e-3, atol=2e-4) if wire == "f32" else dict(rtol=3e-2, atol=3e-3)
    for a, b in zip(losses, ref):
        assert abs(a - b) <= tol["rtol"] * abs(b) + 1e-4, (losses, ref)
    for a, w in zip(ws, m.trainable_variables):
        torch.testing.assert_close(torch.from_numpy(a), w.detach().float().cpu(), **tol)


_MIRRORED_SCRIPT = r'''
import os, sys
sys.path.insert(0, {root!r})
sys.path.insert(0, {tests!r})
import numpy as np
import torch
from distributed_tensorflow_amd import parallel
s = parallel.MirroredStrategy(["GPU:0", "GPU:0"])  # the parent re-runs this script once per device and exits here
import test_dp_gpu as T
rank, world = s.worker_index, s.num_replicas_in_sync
assert world == 2 and s.device == torch.device("cuda", 0)
with s.scope():
    m = T._gpt2(100 + rank)
per = 8 // world
for x, y in T._batches("gpt2", s.device):
    sl = slice(rank * per, (rank + 1) * per)
    m.train_step((x[sl], y[sl]))
torch.cuda.synchronize()
if rank == 0:
    np.savez({out!r}, *[w.detach().float().cpu().numpy() for w in m.trainable_variables])
s.barrier()
'''


def test_mirrored_strategy_over_gpu_list_spawns_one_process_per_device(cuda, tmp_path):
    """MirroredStrategy(["GPU:0", "GPU:0"]): the constructor re-runs the program once per listed
    device, each a rank of the multi-process strategy (two replicas sharing GPU 0 over gloo here; one GPU each on a
    node), and the parent exits with their status. Its weights equal the same 2-rank run under an external launcher
    bitwise, and single-process training within the usual data-parallel rounding."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = str(tmp_path / "w.npz")
    script = tmp_path / "mirrored_run.py"
    script.write_text(_MIRRORED_SCRIPT.format(root=root, tests=os.path.join(root, "tests"), out=out))
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    env["DTF_COLLECTIVE_BACKEND"] = "gloo"
    r = subprocess.run([sys.executable, str(script)], env=env, timeout=300)
    assert r.returncode == 0
    got = np.load(out)
    got = [got[f"arr_{i}"] for i in range(len(got.files))]
    ref = _run_ranks("gpt2")
    for a, b in zip(got, ref[0][1]):
        assert (a == b).all(), "MirroredStrategy(devices) differs from the launcher-started 2-rank run"
    m = _gpt2(100)
    for x, y in _batches("gpt2", cuda):
        m.train_step((x, y))
    torch.cuda.synchronize()
    for a, w in zip(got, m.trainable_variables):
        torch.testing.assert_close(torch.from_numpy(a), w.detach().float().cpu(), rtol=2e-3, atol=2e-4)
