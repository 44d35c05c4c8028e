#!/usr/bin/env python
"""4-wave 256x256 GEMM (gemm4w.hip) vs the current automatic choice (ops.gemm: gemm256 / 128x128 kernels) vs
hipBLASLt, bf16 at square sizes and the BERT-base / GPT-2-medium layer GEMMs (fwd, dX, dW), and fp8 (e4m3 x e4m3 /
e5m2 x e4m3) at the GPT-2-medium projection shapes vs dtf_gemm_fp8_ex and hipBLASLt fp8.

    python tools/bench_gemm4w.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_tensorflow_amd import ops  # noqa: E402
from distributed_tensorflow_amd.ops import fp8 as F  # noqa: E402
from distributed_tensorflow_amd.ops._util import call, ptr, stream  # noqa: E402
from tools.bench_kernels import timeit  # noqa: E402

BF = torch.bfloat16


def g4(a, b, c, M, N, K, ak, bk, out_f32=0, fp8=0, sc=None):
    call("dtf_gemm4w", ptr(a), ptr(b), ptr(c), M, N, K, a.stride(0), b.stride(0), c.stride(0), ak, bk, out_f32, fp8,
         ptr(sc), stream())


def main():
    dev = torch.device("cuda")
    for n in (4096, 8192):
        a = torch.randn(n, n, device=dev).to(BF)
        b = torch.randn(n, n, device=dev).to(BF)
        c = torch.empty(n, n, device=dev, dtype=BF)
        fl = 2.0 * n ** 3
        t4 = timeit(lambda: g4(a, b, c, n, n, n, 0, 0))
        ta = timeit(lambda: ops.gemm(a, b))
        tb = timeit(lambda: a @ b.t())
        print(f"bf16 {n}^3 NT: gemm4w {fl / t4 / 1e12:6.0f} TF | auto {fl / ta / 1e12:6.0f} TF | hipBLASLt "
              f"{fl / tb / 1e12:6.0f} TF", flush=True)
    tot = {"g4": 0.0, "auto": 0.0}
    for T, din, dout in [(16384, 768, 2304), (16384, 768, 768), (16384, 768, 3072), (16384, 3072, 768),
                         (8192, 1024, 3072), (8192, 1024, 1024), (8192, 1024, 4096), (8192, 4096, 1024)]:
        x = torch.randn(T, din, device=dev).to(BF)
        w = torch.randn(dout, din, device=dev).to(BF)
        dy = torch.randn(T, dout, device=dev).to(BF)
        y = torch.empty(T, dout, device=dev, dtype=BF)
        dx = torch.empty(T, din, device=dev, dtype=BF)
        dw = torch.empty(dout, din, device=dev, dtype=torch.float32)
        fl = 2.0 * T * din * dout
        cases = {
            "fwd": (lambda: g4(x, w, y, T, dout, din, 0, 0), lambda: ops.gemm(x, w)),
            "dX": (lambda: g4(dy, w, dx, T, din, dout, 0, 1), lambda: ops.gemm(dy, w, b_kouter=True)),
            "dW": (lambda: g4(dy, x, dw, dout, din, T, 1, 1, 1),
                   lambda: ops.gemm(dy, x, a_kouter=True, b_kouter=True, out_dtype=torch.float32)),
        }
        for name, (f4, fa) in cases.items():
            t4, ta = timeit(f4), timeit(fa)
            tot["g4"] += t4
            tot["auto"] += ta
            print(f"bf16 {name:3s} T={T} {din}->{dout}: gemm4w {t4 * 1e6:6.1f}us {fl / t4 / 1e12:5.0f} TF | auto "
                  f"{ta * 1e6:6.1f}us {fl / ta / 1e12:5.0f} TF ({ta / t4:4.2f}x)", flush=True)
    print({k: round(v * 1e3, 3) for k, v in tot.items()}, "ms (bf16 layer GEMMs)")
    sc = torch.ones(2, device=dev)
    tot = {"g4": 0.0, "cur": 0.0}
    for name, kin, kout in [("qkv", 1024, 3072), ("out", 1024, 1024), ("ffn1", 1024, 4096), ("ffn2", 4096, 1024)]:
        T = 8192
        xq = torch.randint(0, 120, (T, kin), dtype=torch.uint8, device=dev)
        wq = torch.randint(0, 120, (kout, kin), dtype=torch.uint8, device=dev)
        wqT = torch.randint(0, 120, (kin, kout), dtype=torch.uint8, device=dev)
        gq = torch.randint(0, 120, (T, kout), dtype=torch.uint8, device=dev)
        gqT = torch.randint(0, 120, (kout, T), dtype=torch.uint8, device=dev)
        xqT = torch.randint(0, 120, (kin, T), dtype=torch.uint8, device=dev)
        y = torch.empty(T, kout, dtype=BF, device=dev)
        dx = torch.empty(T, kin, dtype=BF, device=dev)
        dw = torch.zeros(kout, kin, dtype=torch.float32, device=dev)
        fl = 2.0 * T * kin * kout
        cases = {
            "fwd": (lambda: g4(xq, wq, y, T, kout, kin, 0, 0, 0, 1, sc), lambda: F.gemm_fp8(xq, wq, sc, y)),
            "dX": (lambda: g4(gq, wqT, dx, T, kin, kout, 0, 0, 0, 2, sc),
                   lambda: F.gemm_fp8(gq, wqT, sc, dx, fmt_a=1)),
            "dW": (lambda: g4(gqT, xqT, dw, kout, kin, T, 0, 0, 1, 2, sc),
                   lambda: F.gemm_fp8(gqT, xqT, sc, dw, fmt_a=1, out_f32=True)),
        }
        for role, (f4, fc) in cases.items():
            t4, tc = timeit(f4), timeit(fc)
            tot["g4"] += t4
            tot["cur"] += tc
            print(f"fp8  {name:4s} {role:3s}: gemm4w {t4 * 1e6:6.1f}us {fl / t4 / 1e12:5.0f} TF | current "
                  f"{tc * 1e6:6.1f}us {fl / tc / 1e12:5.0f} TF ({tc / t4:4.2f}x)", flush=True)
    print({k: round(v * 1e3, 3) for k, v in tot.items()}, "ms (fp8 projection GEMMs, one layer)")


if __name__ == "__main__":
    main()
