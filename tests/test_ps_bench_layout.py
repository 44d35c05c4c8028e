"""bench.py --model resnet50_ps (BASELINE.json config #4): the task-to-GPU layout the launcher gives
2 PS + 6 trainers on an 8-GPU node — one task per GPU, each binding its own device — checked on the CPU with a faked
device count; the 1-GPU rehearsal layout; and the bench entry on a GPU box."""
import json
import os
import subprocess
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_plan_and_layout_8_gpus_one_task_per_gpu():
    from distributed_tensorflow_amd.cli import ps_bench
    n_ps, n_tr = ps_bench.plan(8)
    assert (n_ps, n_tr) == (2, 6)
    lay = ps_bench.layout(8, n_ps, n_tr)
    assert set(lay) == {"ps0", "ps1", "master0"} | {f"worker{i}" for i in range(5)}
    assert sorted(int(v) for v in lay.values()) == list(range(8))  # every GPU once, nobody shares
    assert lay["ps0"] == "0" and lay["ps1"] == "1" and lay["master0"] == "2"


def test_plan_and_layout_other_sizes():
    from distributed_tensorflow_amd.cli import ps_bench
    assert ps_bench.plan(1) == (1, 3)                       # the 1-GPU rehearsal: everything on cuda:0
    assert set(ps_bench.layout(1, 1, 3).values()) == {"0"}
    assert ps_bench.plan(4) == (1, 3) and ps_bench.plan(2) == (1, 1)
    assert ps_bench.plan(8, ps_cpu=True) == (1, 8)
    lay = ps_bench.layout(8, 1, 8, ps_cpu=True)             # host PS: no GPU, trainers take all 8
    assert lay["ps0"] is None and sorted(int(v) for k, v in lay.items() if k != "ps0") == list(range(8))
    with pytest.raises(SystemExit):
        ps_bench.plan(1, ps=1, trainers=0)


def test_each_task_binds_its_own_gpu_with_faked_device_count(monkeypatch):
    """What every task does with its DTF_DEVICE_ORDINAL on an 8-GPU node: context.default_device() is cuda:<ordinal>
    (device count faked to 8; no HIP call is made)."""
    from distributed_tensorflow_amd import context
    from distributed_tensorflow_amd.cli import ps_bench
    monkeypatch.setattr(torch.cuda, "is_available", lambda: True)
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 8)
    monkeypatch.delenv("LOCAL_RANK", raising=False)
    seen = {}
    for role, ordinal in ps_bench.layout(8, *ps_bench.plan(8)).items():
        monkeypatch.setenv("DTF_DEVICE_ORDINAL", ordinal)
        seen[role] = context.default_device()
    assert len(set(seen.values())) == 8 and all(d.type == "cuda" for d in seen.values())


def test_result_line_is_forwarded_unprefixed(capsys):
    from distributed_tensorflow_amd.cli import ps_bench
    tee = ps_bench._Tee()
    tee.write("[worker0] step 1\n[master0] {\"metric\": \"m\", \"value\": 1}\n[ps0] done\n")
    out, err = capsys.readouterr()
    assert out == "{\"metric\": \"m\", \"value\": 1}\n" and "[worker0] step 1" in err and "[ps0] done" in err
    assert json.loads(tee.result)["value"] == 1


@pytest.mark.gpu
def test_bench_ps_one_gpu_prints_one_json_line(tmp_path):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--model", "resnet50_ps", "--gpus", "1",
                        "--steps", "2", "--warmup", "1", "--batch", "16", "--ps-timeout", "400"], cwd=tmp_path,
                       capture_output=True, text=True, timeout=500)
    assert r.returncode == 0, (r.stdout + r.stderr)[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-3000:]
    out = json.loads(lines[0])
    assert out["value"] > 0 and out["n_gpus"] == 1 and out["config"]["ps_tasks"] == 1
    assert out["config"]["trainers"] == 3 and out["config"]["ipc_peer_path"] is True
