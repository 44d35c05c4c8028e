"""ParameterServerStrategy's intra-node data plane on a real GPU (gpurun, one MI355X): PS shards in HBM exported
with HIP IPC, trainers copying gradients into their inboxes and parameters back out (hipMemcpyAsync on IPC-mapped
memory), the native shared-memory mailbox carrying the requests (parallel/ps_shm.py). Every task of the cluster
shares GPU 0 here (same-device IPC across processes); on an 8-GPU node the same copies cross xGMI.

Also the mixed layout the r1 advisor flagged (GPU trainers + CPU PS, DTF_PS_TRANSPORT unset): the chief's
negotiated transport is used by every task, so nobody waits on a rendezvous the others never publish."""
import json
import os
import re
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(tmp_path, ps_gpus, workers=1):
    env = dict(os.environ)
    env.pop("DTF_PS_TRANSPORT", None)
    env["PYTHONPATH"] = ROOT
    cmd = [sys.executable, "-m", "distributed_tensorflow_amd.cli.launch", "--ps", "2", "--workers", str(workers),
           "--chief", "1", "--gpus", "0", "--timeout", "150"] + (["--ps_gpus"] if ps_gpus else []) + \
          ["--", sys.executable, "-m", "distributed_tensorflow_amd.cli.train", "--seed=0", "--max_epochs=3",
           "--optimizer=sgd", "--learning_rate=0.01", "--device=auto"]
    r = subprocess.run(cmd, cwd=tmp_path, env=env, capture_output=True, text=True, timeout=170)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    return out


def test_ps_shards_in_hbm_ipc_data_plane(cuda, tmp_path):
    out = _run(tmp_path, ps_gpus=True, workers=2)
    assert out.count("PS data plane: shm") == 5
    applied = [int(m) for m in re.findall(r"PS applied (\d+) updates", out)]
    assert applied == [3 * 3 * 100] * 2, applied
    w, b = re.findall(r"\[master0\] Get the model, w: ([-\d.e]+), b: ([-\d.e]+)", out)[0]
    assert 1.5 < float(w) < 2.5 and 9.0 < float(b) < 10.5, (w, b)


def test_gpu_trainers_with_cpu_ps_negotiate_one_transport(cuda, tmp_path):
    out = _run(tmp_path, ps_gpus=False)
    assert out.count("PS data plane: shm") == 4
    assert "Exported SavedModel" in out


def _overlap_cluster(tmp_path, trainers, overlap, staleness="0", steps=20):
    env = dict(os.environ, PYTHONPATH=ROOT, DTF_PS_OVERLAP="1" if overlap else "0", DTF_PS_STALENESS=staleness,
               PS_TEST_STEPS=str(steps))
    env.pop("DTF_PS_TRANSPORT", None)
    cmd = [sys.executable, "-m", "distributed_tensorflow_amd.cli.launch", "--ps", "1", "--workers",
           str(trainers - 1), "--chief", "1", "--gpus", "0", "--ps_gpus", "--host_kv", "--timeout", "150", "--",
           sys.executable, "-m", "tests.tasks.ps_overlap_task"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=170)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    res = [json.loads(m) for m in re.findall(r"PSTEST (\{.*\})", out)]
    assert len(res) == trainers, out[-3000:]
    return res


def test_ps_push_overlap_applies_every_push_once_and_matches_unoverlapped(cuda, tmp_path):
    """PSPushBucketer: GPU trainers copy gradient buckets into the PS inboxes during backward. One
    trainer: the overlapped and the plain push must give bit-identical PS parameters (same pushes, same order);
    two trainers: every push is applied exactly once (the PS global_step counts them all)."""
    a = _overlap_cluster(tmp_path, 1, overlap=True)[0]
    b = _overlap_cluster(tmp_path, 1, overlap=False)[0]
    assert a["overlap_push"] and not b["overlap_push"]
    assert a["global_step"] == b["global_step"] == 20
    assert a["checksum"] == b["checksum"], (a, b)
    two = _overlap_cluster(tmp_path, 2, overlap=True, staleness="1")
    assert all(t["overlap_push"] and t["staleness"] == 1 for t in two)
    assert all(t["global_step"] == 40 for t in two), two
