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
    out = bench._allreduce_sweep(dist, torch.device("cpu"), world, sizes_mb=(1, 2), iters=2)
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
    assert set(res[0]) == {"1MB", "2MB"} and res[0] == res[1]
    assert all(v > 0 for v in res[0].values())
