"""Correctness + speed of the 256x256 glds GEMM vs the 128x128 kernel and hipBLASLt (torch.matmul)."""
import sys
import time

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from distributed_tensorflow_amd import ops  # noqa: E402
from distributed_tensorflow_amd.ops._util import call, ptr, stream  # noqa: E402


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters


def g256(a, b, out):
    M, K = a.shape
    N = b.shape[0]
    call("dtf_gemm256", ptr(a), ptr(b), ptr(out), M, N, K, K, K, N, int(out.dtype == torch.float32), stream())
    return out


dev = torch.device("cuda")
torch.manual_seed(0)
ok = True
for (M, N, K) in [(256, 256, 128), (300, 260, 192), (1000, 777 // 4 * 4, 640), (4096, 4096, 4096), (8192, 8192, 8192),
                  (16384, 768, 768), (16384, 3072, 768), (16384, 768, 3072), (16384, 2304, 768), (8192, 4096, 1024),
                  (8192, 1024, 4096), (8192, 3072, 1024)]:
    a = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
    b = (torch.rand(N, K, device=dev) * 2 - 1).to(torch.bfloat16)
    out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    g256(a, b, out)
    ref = a.float() @ b.float().t()
    err = (out.float() - ref).abs().max().item() / (ref.abs().max().item() + 1e-6)
    good = err < 2e-2
    ok &= good
    fl = 2.0 * M * N * K
    t1 = timeit(lambda: g256(a, b, out))
    t2 = timeit(lambda: ops.gemm(a, b))
    t3 = timeit(lambda: a @ b.t())
    print(f"{M:6d}x{N:5d}x{K:5d} err={err:.2e} {'OK ' if good else 'BAD'} "
          f"g256 {fl / t1 / 1e12:7.1f} TF  g128 {fl / t2 / 1e12:7.1f} TF  hipblaslt {fl / t3 / 1e12:7.1f} TF", flush=True)
print("ALL OK" if ok else "FAILURES")
sys.exit(0 if ok else 1)
