"""Correctness + speed of the 256x256 glds GEMM (all operand layouts, split-K) vs the 128x128 kernel and
hipBLASLt (torch.matmul). Shapes are the BERT-base / GPT-2-medium projection GEMMs and squares."""
import sys
import time

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from distributed_tensorflow_amd import ops  # noqa: E402
from distributed_tensorflow_amd.ops._util import call, ptr, stream, workspace  # noqa: E402


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters


def g256(a, b, out, ak, bk, splitk=1):
    M, N = out.shape
    K = a.shape[0] if ak else a.shape[1]
    ws = workspace(out.device)
    rc = call("dtf_gemm256", ptr(a), ptr(b), ptr(out), M, N, K, a.shape[1], b.shape[1], N, int(ak), int(bk),
              int(out.dtype == torch.float32), splitk, ptr(ws), ws.numel(), stream())
    return out


dev = torch.device("cuda")
torch.manual_seed(0)
ok = True
shapes = [(304, 264, 192), (4096, 4096, 4096), (8192, 8192, 8192), (16384, 768, 768), (16384, 3072, 768),
          (16384, 768, 3072), (16384, 2304, 768), (8192, 4096, 1024), (8192, 1024, 4096), (8192, 3072, 1024)]
for (M, N, K) in shapes:
    for layout in ("NT", "NN", "TN"):
        ak, bk = layout == "TN", layout in ("NN", "TN")
        a = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
        b = (torch.rand(N, K, device=dev) * 2 - 1).to(torch.bfloat16)
        A = a.t().contiguous() if ak else a
        B = b.t().contiguous() if bk else b
        f32 = layout == "TN"
        out = torch.empty(M, N, device=dev, dtype=torch.float32 if f32 else torch.bfloat16)
        sk = 1
        if layout == "TN":  # weight-gradient shapes: few tiles, long K -> split
            t = ((M + 255) // 256) * ((N + 255) // 256)
            sk = max(1, min(-(-256 // t), K // 1024))
        g256(A, B, out, ak, bk, sk)
        ref = a.float() @ b.float().t()
        err = (out.float() - ref).abs().max().item() / (ref.abs().max().item() + 1e-6)
        good = err < 2e-2
        ok &= good
        fl = 2.0 * M * N * K
        t1 = timeit(lambda: g256(A, B, out, ak, bk, sk))
        t2 = timeit(lambda: ops.gemm(A, B, a_kouter=ak, b_kouter=bk, out_dtype=out.dtype, tile=0))
        t3 = timeit(lambda: a @ b.t())
        print(f"{layout} {M:6d}x{N:5d}x{K:5d} sk={sk} err={err:.1e} {'OK ' if good else 'BAD'} "
              f"g256 {fl / t1 / 1e12:7.1f} TF  g128 {fl / t2 / 1e12:7.1f} TF  hipblaslt {fl / t3 / 1e12:7.1f} TF",
              flush=True)
print("ALL OK" if ok else "FAILURES")
sys.exit(0 if ok else 1)
