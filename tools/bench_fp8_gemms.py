#!/usr/bin/env python
"""FP8 vs bf16 GEMMs at the GPT-2-medium projection shapes (8 x 1024 tokens; QKV, attention out, FFN1, FFN2), each in
its three roles: forward (x W^T), data gradient (dZ W) and weight gradient (dZ^T X over the tokens). bf16 through
ops.gemm's automatic kernel choice; fp8 through dtf_gemm_fp8_ex (e4m3 x e4m3 forward, e5m2 x e4m3 backward, the
operand layouts ops/fp8.py hands it); hipBLASLt fp8 (torch._scaled_mm) for reference when this torch has it; and
the transposing quantize pass (ops.fp8.quantize_t) that feeds each fp8 GEMM.

    python tools/bench_fp8_gemms.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_tensorflow_amd import ops  # noqa: E402
from distributed_tensorflow_amd.ops import fp8 as F  # noqa: E402
from tools.bench_kernels import timeit  # noqa: E402

BF = torch.bfloat16
SHAPES = [("qkv", 1024, 3072), ("out", 1024, 1024), ("ffn1", 1024, 4096), ("ffn2", 4096, 1024)]


def main():
    dev = torch.device("cuda")
    T = 8192
    sc = torch.ones(2, device=dev)
    tot = {"bf16": 0.0, "fp8": 0.0, "fp8_8wave": 0.0, "quant": 0.0}
    for name, kin, kout in SHAPES:
        x = torch.randn(T, kin, device=dev).to(BF)
        w = (torch.randn(kout, kin, device=dev) * 0.05).to(BF)
        dz = torch.randn(T, kout, device=dev).to(BF)
        xq = torch.randint(0, 120, (T, kin), dtype=torch.uint8, device=dev)      # e4m3 bytes (finite)
        wq = torch.randint(0, 120, (kout, kin), dtype=torch.uint8, device=dev)
        wqT = torch.randint(0, 120, (kin, kout), dtype=torch.uint8, device=dev)
        gq = torch.randint(0, 120, (T, kout), dtype=torch.uint8, device=dev)     # e5m2 bytes
        gqT = torch.randint(0, 120, (kout, T), dtype=torch.uint8, device=dev)
        xqT = torch.randint(0, 120, (kin, T), dtype=torch.uint8, device=dev)
        y = torch.empty(T, kout, dtype=BF, device=dev)
        dx = torch.empty(T, kin, dtype=BF, device=dev)
        dw = torch.zeros(kout, kin, dtype=torch.float32, device=dev)
        roles = {
            "fwd": (lambda: ops.gemm(x, w), lambda: F.gemm_fp8(xq, wq, sc, y)),
            "dX": (lambda: ops.gemm(dz, w, b_kouter=True), lambda: F.gemm_fp8(gq, wqT, sc, dx, fmt_a=1)),
            "dW": (lambda: ops.gemm(dz, x, a_kouter=True, b_kouter=True, out_dtype=torch.float32),
                   lambda: F.gemm_fp8(gqT, xqT, sc, dw, fmt_a=1, out_f32=True, beta=1.0)),
        }
        from distributed_tensorflow_amd._native import kernels
        for role, (fb, f8) in roles.items():
            fl = 2.0 * T * kin * kout
            tb = timeit(fb)
            kernels().dtf_fp8_w4_enable(0)
            t8o = timeit(f8)
            kernels().dtf_fp8_w4_enable(-1)
            t8 = timeit(f8)
            tot["bf16"] += tb
            tot["fp8"] += t8
            tot["fp8_8wave"] += t8o
            line = (f"{name:4s} {role:3s} T={T} {kin}->{kout}: bf16 {tb * 1e6:6.1f}us {fl / tb / 1e12:6.0f} TF | "
                    f"fp8 4-wave {t8 * 1e6:6.1f}us {fl / t8 / 1e12:6.0f} TF ({tb / t8:4.2f}x bf16) | "
                    f"fp8 8-wave {t8o * 1e6:6.1f}us {fl / t8o / 1e12:6.0f} TF")
            if hasattr(torch, "_scaled_mm") and hasattr(torch, "float8_e4m3fn") and role == "fwd":
                try:
                    a8 = x.to(torch.float8_e4m3fn)
                    b8 = w.to(torch.float8_e4m3fn)
                    one = torch.ones((), device=dev)
                    tl = timeit(lambda: torch._scaled_mm(a8, b8.t(), scale_a=one, scale_b=one, out_dtype=BF))
                    line += f" | hipBLASLt fp8 {tl * 1e6:6.1f}us {fl / tl / 1e12:6.0f} TF"
                except Exception as e:  # noqa: BLE001
                    line += f" | hipBLASLt fp8 n/a ({type(e).__name__})"
            print(line, flush=True)
        # the quantize passes feeding them: activation (e4m3, row-major + transposed) and gradient (e5m2)
        s = torch.ones(1, device=dev)
        am = torch.zeros(1, device=dev)
        tq = timeit(lambda: F.quantize_t(x, s, am, fmt=0))
        tg = timeit(lambda: F.quantize_t(dz, s, am, fmt=1, rowmajor=True))
        tot["quant"] += tq + tg
        print(f"{name:4s} quantize: x [{T},{kin}] e4m3 (+T) {tq * 1e6:6.1f}us  dZ [{T},{kout}] e5m2 (+T) "
              f"{tg * 1e6:6.1f}us", flush=True)
    print({k: round(v * 1e3, 3) for k, v in tot.items()}, "ms per layer (fwd + dX + dW of the 4 projections)")
    # the two producer-quantizing GEMMs of a block (dtf_gemm_fp8_q8): FFN1 forward (GELU, pre-activation side output,
    # e4m3 copy + transpose of the output for FFN2) and FFN2's data gradient (GELU backward, e5m2 copy + transpose +
    # bias-gradient column sums for FFN1)
    from distributed_tensorflow_amd.ops._util import K as KL, ptr, stream
    from distributed_tensorflow_amd._native import kernels
    buf = torch.tensor([1.0, 0.0, 1.0, 0.0, 0.0], device=dev)
    for name, M, N, Kd, fmt_a, dact in (("ffn1 fwd q8", T, 4096, 1024, 0, 0), ("ffn2 dX q8", T, 1024, 4096, 1, 2)):
        a = torch.randint(0, 120, (M, Kd), dtype=torch.uint8, device=dev)
        b = torch.randint(0, 120, (N, Kd), dtype=torch.uint8, device=dev)
        aux = torch.empty(M, N, dtype=BF, device=dev)
        pre = torch.randn(M, N, device=dev).to(BF)
        bias = torch.zeros(N, device=dev)
        q = torch.empty(M, N, dtype=torch.uint8, device=dev)
        qT = torch.empty(N, M, dtype=torch.uint8, device=dev)
        cp = torch.empty(M // 128, N, dtype=torch.float32, device=dev)

        def f():
            rc = KL().dtf_gemm_fp8_q8(ptr(a), ptr(b), None, ptr(aux) if not dact else None,
                                      ptr(bias) if not dact else None, ptr(sc), M, N, Kd, Kd, Kd, 0 if dact else 2,
                                      fmt_a, ptr(pre) if dact else None, dact, None, ptr(q), ptr(qT),
                                      ptr(cp) if dact else None, fmt_a, ptr(buf[0:1]), ptr(buf[1:2]), ptr(buf[2:3]),
                                      ptr(buf[3:4]), ptr(buf[4:5]), stream())
            assert rc == 0, rc
        kernels().dtf_fp8_w4_enable(0)
        to = timeit(f)
        kernels().dtf_fp8_w4_enable(1)
        t4 = timeit(f)
        kernels().dtf_fp8_w4_enable(-1)
        fl = 2.0 * M * N * Kd
        print(f"{name}: 4-wave {t4 * 1e6:6.1f}us {fl / t4 / 1e12:6.0f} TF | 8-wave {to * 1e6:6.1f}us "
              f"{fl / to / 1e12:6.0f} TF", flush=True)


if __name__ == "__main__":
    main()
