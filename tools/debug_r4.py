"""Bisect harness for two round-4 GPU mismatches (run on the GPU box).

  python tools/debug_r4.py capture   # captured vs eager overlapped update, with variants
  python tools/debug_r4.py p2p       # 2-rank GPT-2 (gloo, ranks share cuda:0): P2P vs gloo buckets vs 1 process
"""
import contextlib
import multiprocessing as mp
import os
import socket
import sys
import traceback

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])


def _small_resnet(seed):
    from distributed_tensorflow_amd.keras import initializers
    from distributed_tensorflow_amd.models import ResNet
    initializers.set_seed(seed)
    return ResNet(50, num_classes=16, width=16)


def capture(variant):
    from distributed_tensorflow_amd.keras import losses, optimizers
    from distributed_tensorflow_amd.ops import _util
    from distributed_tensorflow_amd.parallel import strategy as S
    S._OVERLAP_UPDATE = "1"
    if variant == "upd_main":
        _util.update_stream_ctx = lambda device, extra_wait=None: contextlib.nullcontext()
    if variant == "defer":  # every bucket update after backward (finalize), none during it
        from distributed_tensorflow_amd.parallel import collective
        collective.GradientBucketer._launch_ready = lambda self: None
    if variant == "sync_upd":  # the update stream also waits for EVERYTHING on main before each bucket update
        real = _util.update_stream_ctx

        def ctx(device, extra_wait=None):
            torch.cuda.current_stream(device).wait_stream(_util.side_stream(device))
            return real(device, extra_wait)
        _util.update_stream_ctx = ctx
    cuda = torch.device("cuda:0")
    torch.manual_seed(0)
    xs = [torch.randn(8, 3, 64, 64, device=cuda) for _ in range(6)]
    ys = [torch.randint(0, 16, (8,), device=cuda) for _ in range(6)]
    outs, snaps = [], []
    for jit in (False, True):
        model = _small_resnet(7)
        o = optimizers.SGD(0.05, momentum=0.9)
        model.compile(optimizer=o, loss=losses.SparseCategoricalCrossentropy(from_logits=True), jit_compile=jit)
        fn = model.make_train_function(force=True)
        ls, sn = [], []
        for x, y in zip(xs, ys):
            ls.append(float(fn((x, y))["loss"]))
            torch.cuda.synchronize()
            sn.append([(w.name, w.detach().float().cpu().clone()) for w in model.weights])
        outs.append(ls)
        snaps.append(sn)
        S.get_strategy()._bucketers.clear()
    print(variant, "eager", [round(v, 4) for v in outs[0]], flush=True)
    print(variant, "graph", [round(v, 4) for v in outs[1]], flush=True)
    print(variant, "MATCH" if all(abs(a - b) < 1e-3 for a, b in zip(*outs)) else "DIFF", flush=True)
    for step, (a, b) in enumerate(zip(*snaps)):
        bad = []
        for (n, wa), (_, wb) in zip(a, b):
            d = float((wa - wb).abs().max())
            if d > 1e-6 + 1e-3 * float(wa.abs().max()):
                bad.append((d, n))
        bad.sort(reverse=True)
        print(f"  after step {step + 1}: {len(bad)}/{len(a)} tensors differ; first in model order: "
              f"{[n for _, n in sorted(bad, key=lambda t: [w[0] for w in a].index(t[1]))[:4]]} worst {bad[:3]}",
              flush=True)


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
    m.compile(optimizer=optimizers.SGD(0.1, momentum=0.9),
              loss=losses.SparseCategoricalCrossentropy(from_logits=True))
    return m


def _batches(dev, steps=3):
    g = torch.Generator().manual_seed(5)
    out = []
    for _ in range(steps):
        ids = torch.randint(0, 320, (8, 128), generator=g)
        out.append((ids.to(dev), torch.roll(ids, -1, 1).to(dev)))
    return out


def _worker(rank, world, port, mode, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port), DTF_COLLECTIVE_BACKEND="gloo", DTF_P2P="0" if mode == "gloo" else "1")
    try:
        import torch.distributed as dist
        from distributed_tensorflow_amd import parallel
        from distributed_tensorflow_amd.parallel import p2p
        orig = p2p.P2PAllReducer.all_reduce_
        from distributed_tensorflow_amd.ops import _util

        def wrapped(self, lo, hi):
            if mode in ("p2p_sync", "p2p_before"):
                torch.cuda.synchronize()
            if mode in ("p2p_sync", "p2p_barrier"):
                dist.barrier()
            orig(self, lo, hi)
            if mode == "p2p_sync":
                torch.cuda.synchronize()
            if mode == "p2p_mainwait":
                torch.cuda.default_stream().wait_stream(torch.cuda.current_stream())
        p2p.P2PAllReducer.all_reduce_ = wrapped
        if mode == "p2p_main":  # issue on the main stream after it joined the side stream
            def ctx_main(device):
                torch.cuda.current_stream(device).wait_stream(_util.side_stream(device))
                return contextlib.nullcontext()
            _util.collective_ctx = ctx_main
        s = parallel.MultiWorkerMirroredStrategy(bucket_mb=0.25)
        with s.scope():
            m = _gpt2(100 + rank)
        grads = []
        per = 8 // world
        b = None
        for x, y in _batches(s.device):
            sl = slice(rank * per, (rank + 1) * per)
            m.train_step((x[sl], y[sl]))
            b = s._bucketers[id(m._arena)]
        torch.cuda.synchronize()
        q.put((rank, [w.detach().float().cpu().numpy() for w in m.trainable_variables],
               [w.name for w in m.trainable_variables], dict(b.paths), (b.buckets, list(m._arena.offsets))))
        dist.barrier()
        dist.destroy_process_group()
    except Exception:
        q.put((rank, None, traceback.format_exc(), None, None))


def run_ranks(mode, world=2):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, mode, q)) for r in range(world)]
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


def p2p_main():
    import numpy as np
    cuda = torch.device("cuda:0")
    m = _gpt2(100)
    for x, y in _batches(cuda):
        m.train_step((x, y))
    torch.cuda.synchronize()
    ref = [w.detach().float().cpu().numpy() for w in m.trainable_variables]
    names = [w.name for w in m.trainable_variables]
    for mode in sys.argv[2:] or ("gloo", "p2p", "p2p_sync"):
        res = run_ranks(mode)
        same = all((a == b).all() for a, b in zip(res[0][1], res[1][1]))
        buckets, offs = res[0][4]
        print(f"{mode}: paths={res[0][3]} replicas_identical={same} buckets={buckets}", flush=True)
        for n, a, r, o in zip(names, res[0][1], ref, offs):
            d = np.abs(a - r)
            bad = (d > 2e-4 + 2e-3 * np.abs(r)).mean()
            if bad > 0:
                bi = [i for i, (lo, hi) in enumerate(buckets) if lo <= o < hi]
                print(f"   {n:40s} shape={a.shape} off={o} bucket={bi} maxdiff={d.max():.3e} frac_bad={bad:.3f}",
                      flush=True)


if __name__ == "__main__":
    what = sys.argv[1]
    if what == "capture":
        for v in sys.argv[2:] or ["base", "upd_main"]:
            capture(v)
    else:
        p2p_main()
