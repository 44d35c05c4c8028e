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


def _worker_skip(rank, world, port, q):
    """Rank 0 reduces a bucket that rank 1 never contributes to: its kernel must give up after the (short) timeout,
    set the error word and raise from check() — no hang."""
    try:
        import time
        import torch.distributed as dist
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from distributed_tensorflow_amd.parallel.p2p import P2PAllReducer
        dev = torch.device("cuda", 0)
        grad = torch.ones(8192, dtype=torch.float32, device=dev)
        red = P2PAllReducer(grad, spans=[(0, 4096), (4096, 8192)])
        raised, took = None, 0.0
        if rank == 0:
            t0 = time.time()
            red.all_reduce_(0, 4096, timeout_ms=2000)
            torch.cuda.synchronize()
            took = time.time() - t0
            try:
                red.check()
                raised = False
            except RuntimeError:
                raised = True
        dist.barrier()
        red.close()
        dist.destroy_process_group()
        q.put((rank, raised, took))
    except Exception:
        q.put((rank, traceback.format_exc(), 0.0))


def test_p2p_peer_skipping_a_call_times_out(cuda):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker_skip, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict((r, (raised, took)) for r, raised, took in (q.get(timeout=150) for _ in ps))
    for p in ps:
        p.join(30)
    raised, took = res[0]
    assert raised is True, raised
    assert took < 60, took


def _worker_producer(rank, world, port, q):
    """The bucket's producer still runs on the weight-gradient side stream (a long sleep, then the write) when the
    bucket is issued: the P2P kernel goes to the communication stream, which waits for the side stream's work issued
    so far (comm_stream_ctx), so it must sum the PRODUCED values."""
    try:
        import torch.distributed as dist
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from distributed_tensorflow_amd.ops import _util
        from distributed_tensorflow_amd.parallel.p2p import P2PAllReducer
        dev = torch.device("cuda", 0)
        grad = torch.zeros(65536, dtype=torch.float32, device=dev)
        red = P2PAllReducer(grad, spans=[(0, 65536)])
        torch.cuda.synchronize()
        dist.barrier()
        with _util.fork_side(dev, grad):
            torch.cuda._sleep(200_000_000)  # ~0.1 s of GPU time before the producer writes
            grad.fill_(float(rank + 1))
        with _util.comm_stream_ctx(dev):
            red.all_reduce_(0, 65536)
        _util.join_side_streams()
        _util.join_comm_stream(dev)
        torch.cuda.synchronize()
        red.check()
        ok = bool((grad == float(world * (world + 1) // 2)).all().item())
        dist.barrier()
        red.close()
        dist.destroy_process_group()
        q.put((rank, ok))
    except Exception:
        q.put((rank, traceback.format_exc()))


def test_p2p_waits_for_a_producer_on_another_stream(cuda):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker_producer, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=150) for _ in ps)
    for p in ps:
        p.join(30)
    assert res[0] is True and res[1] is True, res
