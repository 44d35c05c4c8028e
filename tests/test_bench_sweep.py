"""bench.py's post-timing all-reduce sweep (reported as allreduce_busbw_GBps by multi-GPU runs) on a 2-rank gloo
group: every size is reported, positive, and identical on both ranks (slowest-rank time)."""
import os
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sys.path.insert(0, ROOT)
    import bench
    out = bench._allreduce_sweep(dist, torch.device("cpu"), world, [], sizes_mb=(1, 2), iters=2)
    q.put((rank, out))
    dist.destroy_process_group()


def test_allreduce_sweep_gloo_world2():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    # no GPU communicator here: only the process-group row (the native rows need the nccl backend)
    assert set(res[0]) == {"torch_process_group"} and res[0] == res[1]
    pg = res[0]["torch_process_group"]
    assert set(pg) == {"1MB", "2MB"} and all(v > 0 for v in pg.values())


@pytest.mark.gpu
def test_bench_multirank_path_on_one_gpu(tmp_path):
    """bench.py's N>1 path end to end, rehearsed on a 1-GPU box: `--gpus 2` relaunches itself
    under torch.distributed.run, both ranks share cuda:0 and reduce over gloo (DTF_COLLECTIVE_BACKEND=gloo; RCCL
    refuses two ranks on one device), and rank 0 prints ONE JSON line with the whole-job value, the world size, the
    cross-rank weight checksum agreement and the all-reduce sweep."""
    import json
    import subprocess
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    env = dict(os.environ, DTF_COLLECTIVE_BACKEND="gloo")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--batch", "32", "--steps",
                        "2", "--warmup", "1"], cwd=tmp_path, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, (r.stdout + r.stderr)[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-3000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["rccl_world"] == 2 and out["process_group_backend"] == "gloo"
    assert out["replicas_identical"] is True
    assert out["config"]["global_batch"] == 64 and out["config"]["parallelism"] == "dp2"
    sweep = out["allreduce_busbw_GBps"]
    assert isinstance(sweep, dict) and len(sweep["torch_process_group"]) == 6
    assert out["value"] > 0 and out["steps"] == 2 and out["warmup"] == 1
