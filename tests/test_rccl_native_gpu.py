"""The framework's own RCCL communicator (csrc/runtime/rccl_comm.cc, parallel/rccl.py) on one MI355X.

RCCL refuses two ranks on one GPU, so the box runs world size 1: that still covers the unique-id exchange through the
rendezvous store, ncclCommInitRankConfig with a channel (CTA) configuration, every collective entry point against its
definition, stream ordering on a non-default stream, hipGraph capture + replay of a collective, and destroy. The
gradient bucketer's use of it is covered by tests/test_dp_gpu.py::test_rccl_bucketer_world1_matches_single_process.
"""
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


def _worker(port, q):
    try:
        import torch.distributed as dist
        from distributed_tensorflow_amd.parallel import rccl
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                                device_id=torch.device("cuda", 0))
        dev = torch.device("cuda", 0)
        comm = rccl.RcclCommunicator(min_channels=8, max_channels=16)   # runs its own self-check
        out = {"version": rccl.version(), "info0": comm.info()}
        g = torch.Generator(device=dev).manual_seed(0)
        x = torch.randn(1 << 20, device=dev, generator=g)
        ref = x.clone()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):  # stream-ordered on the caller's stream
            comm.all_reduce_(x)
            x.mul_(3)
        torch.cuda.current_stream().wait_stream(s)
        out["allreduce_f32"] = bool(torch.equal(x, ref * 3))
        xb = ref.to(torch.bfloat16)
        out["allreduce_bf16_max"] = bool(torch.equal(comm.all_reduce_(xb.clone(), op="max"), xb))
        rs = torch.empty(1 << 20, device=dev)
        out["reduce_scatter"] = bool(torch.equal(comm.reduce_scatter(ref, rs), ref))
        ag = torch.empty(1 << 20, device=dev)
        out["all_gather"] = bool(torch.equal(comm.all_gather(ref, ag), ref))
        out["broadcast"] = bool(torch.equal(comm.broadcast_(ref.clone(), root=0), ref))
        # self send/recv in one group
        r = torch.zeros(4096, device=dev)
        comm.group_start()
        comm.send(ref[:4096], 0)
        comm.recv(r, 0)
        comm.group_end()
        out["sendrecv"] = bool(torch.equal(r, ref[:4096]))
        # hipGraph capture of a collective between two kernels, replayed 3 times
        t = torch.ones(4096, device=dev)
        torch.cuda.synchronize()
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr):
            t.mul_(2)
            comm.all_reduce_(t)
            t.add_(1)
        t.fill_(1.0)
        for _ in range(3):
            gr.replay()
        torch.cuda.synchronize()
        out["graph"] = float(t[0].item())   # ((1*2+1)*2+1)*2+1 = 15
        out["async_error"] = comm.async_error()
        out["info1"] = comm.info()
        comm.destroy()
        dist.destroy_process_group()
        q.put(out)
    except Exception:
        q.put({"error": traceback.format_exc()})


def test_native_rccl_communicator_world1(cuda):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker, args=(_port(), q))
    p.start()
    try:
        out = q.get(timeout=120)
    finally:
        p.join(30)
        if p.is_alive():
            p.kill()
    assert "error" not in out, out.get("error")
    assert out["version"] >= 22000
    assert out["info0"]["nranks"] == 1 and out["info0"]["min_channels"] == 8 and out["info0"]["max_channels"] == 16
    for k in ("allreduce_f32", "allreduce_bf16_max", "reduce_scatter", "all_gather", "broadcast", "sendrecv"):
        assert out[k], k
    assert out["graph"] == 15.0, out["graph"]
    assert out["async_error"] == 0
    assert out["info1"]["calls"] >= 9 and out["info1"]["bytes"] > (1 << 22), out["info1"]
