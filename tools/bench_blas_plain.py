"""Plain (epilogue-free) GEMMs of the transformer backward passes: our MFMA kernel (ops.gemm) vs hipBLASLt
(torch.mm / addmm with f32 output). dgrad: dX[T,in] = dZ[T,out] W[out,in] (bf16 out); wgrad: dW[out,in] +=
dZ^T X (f32 accumulate into the gradient arena).

  python tools/bench_blas_plain.py
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
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
torch.manual_seed(0)
BF = torch.bfloat16
for (T, o, i) in [(16384, 2304, 768), (16384, 768, 768), (16384, 3072, 768), (16384, 768, 3072),
                  (8192, 3072, 1024), (8192, 1024, 1024), (8192, 4096, 1024), (8192, 1024, 4096),
                  (8192, 50304, 1024)]:
    dz = torch.randn(T, o, device=dev).to(BF)
    x = torch.randn(T, i, device=dev).to(BF)
    w = torch.randn(o, i, device=dev).to(BF)
    dw = torch.zeros(o, i, device=dev)
    fl = 2.0 * T * o * i
    t1 = timeit(lambda: ops.gemm(dz, w, b_kouter=True))
    t2 = timeit(lambda: torch.mm(dz, w))
    t3 = timeit(lambda: ops.gemm(dz, x, a_kouter=True, b_kouter=True, out=dw, beta=1.0))
    t4 = timeit(lambda: dw.add_(torch.mm(dz.t(), x, out_dtype=torch.float32)))
    try:
        t5 = timeit(lambda: torch.ops.aten.addmm.dtype_out(dw, dz.t(), x, torch.float32, beta=1, alpha=1, out=dw))
    except Exception as e:  # noqa: BLE001
        t5 = float("nan")
        print("addmm dtype_out:", e)
    ref = (dz.float().t() @ x.float())
    dw.zero_()
    torch.ops.aten.addmm.dtype_out(dw, dz.t(), x, torch.float32, beta=1, alpha=1, out=dw)
    err = ((dw - ref).abs().max() / ref.abs().max()).item()
    print(f"T={T:6d} out={o:6d} in={i:5d}  dgrad ours {fl / t1 / 1e12:6.0f} TF  blas {fl / t2 / 1e12:6.0f} TF | "
          f"wgrad ours {fl / t3 / 1e12:6.0f} TF  blas mm+add {fl / t4 / 1e12:6.0f} TF  blas addmm {fl / t5 / 1e12:6.0f}"
          f" TF (err {err:.1e})", flush=True)
