"""The GEMMs of one BERT-base / GPT-2-medium layer step (fwd, dX, dW) through ops.gemm's automatic kernel
choice vs the 128x128 kernel forced, vs hipBLASLt."""
import sys
import time

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from distributed_tensorflow_amd import ops  # noqa: E402


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters


dev = torch.device("cuda")
tot = {"auto": 0.0, "g128": 0.0, "blas": 0.0}
for T, d_in, d_out in [(16384, 768, 2304), (16384, 768, 768), (16384, 768, 3072), (16384, 3072, 768),
                       (8192, 1024, 3072), (8192, 1024, 1024), (8192, 1024, 4096), (8192, 4096, 1024)]:
    x = torch.randn(T, d_in, device=dev).to(torch.bfloat16)
    w = torch.randn(d_out, d_in, device=dev).to(torch.bfloat16)
    dy = torch.randn(T, d_out, device=dev).to(torch.bfloat16)
    cases = {
        "fwd": (lambda tile: ops.gemm(x, w, tile=tile), lambda: x @ w.t()),
        "dX": (lambda tile: ops.gemm(dy, w, b_kouter=True, tile=tile), lambda: dy @ w),
        "dW": (lambda tile: ops.gemm(dy, x, a_kouter=True, b_kouter=True, out_dtype=torch.float32, tile=tile),
               lambda: dy.t() @ x),
    }
    for name, (f, ref) in cases.items():
        fl = 2.0 * T * d_in * d_out
        ta, tg, tb = timeit(lambda: f(-1)), timeit(lambda: f(0)), timeit(ref)
        tot["auto"] += ta
        tot["g128"] += tg
        tot["blas"] += tb
        print(f"{name:3s} T={T} {d_in}->{d_out}: auto {fl / ta / 1e12:6.1f} TF  g128 {fl / tg / 1e12:6.1f} TF  "
              f"hipblaslt {fl / tb / 1e12:6.1f} TF", flush=True)
print({k: round(v * 1e3, 3) for k, v in tot.items()}, "ms total")
