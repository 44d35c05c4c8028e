"""The one-shot P2P all-reduce (parallel/p2p.py, csrc/kernels/p2p_allreduce.hip) with 2 and 4 ranks sharing GPU 0:
the ranks map each other's gradient arenas and flag arrays through HIP IPC handles (the mechanism the PS data plane
uses across processes, tests/test_ps_gpu.py) and exchange them over a gloo group; on an 8-GPU node the same
mappings cross xGMI. Every call must leave EVERY rank holding exactly the f32 sum taken in rank order
(x0 + x1 + ... bitwise), including the float4 tail handling and consecutive calls on other ranges (epochs)."""
import multiprocessing as mp
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


def _data(rank, n, call):
    g = torch.Generator().manual_seed(1000 * call + rank)
    return torch.randn(n, generator=g)


CALLS = [(0, 4096), (17, 100003), (4096, 4096 + 262144), (5, 9)]  # [lo, hi) per call


def _worker(rank, world, port, n, q):
    try:
        import torch.distributed as dist
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from distributed_tensorflow_amd.parallel.p2p import P2PAllReducer
        dev = torch.device("cuda", 0)
        grad = torch.zeros(n, dtype=torch.float32, device=dev)
        red = P2PAllReducer(grad)
        ok = []
        for c, (lo, hi) in enumerate(CALLS):
            grad[lo:hi].copy_(_data(rank, hi - lo, c).to(dev))  # stream-ordered before the kernel: no barrier
            red.all_reduce_(lo, hi)
            torch.cuda.synchronize()
            red.check()
            exp = _data(0, hi - lo, c)
            for p in range(1, world):
                exp = exp + _data(p, hi - lo, c)
            ok.append(bool(torch.equal(grad[lo:hi].cpu(), exp)))
        dist.barrier()
        red.close()
        dist.destroy_process_group()
        q.put((rank, ok, red.calls))
    except Exception:
        q.put((rank, traceback.format_exc(), 0))


@pytest.mark.parametrize("world", [2, 4])
def test_p2p_allreduce_matches_ordered_sum(cuda, world):
    n = 4096 + 262144 + 64
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict((r, (ok, calls)) for r, ok, calls in (q.get(timeout=150) for _ in ps))
    for p in ps:
        p.join(30)
    for r in range(world):
        ok, calls = res[r]
        assert isinstance(ok, list), ok
        assert all(ok), (r, ok)
        assert calls == len(CALLS)
