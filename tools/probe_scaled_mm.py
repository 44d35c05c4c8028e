"""hipBLASLt fp8 (torch._scaled_mm) at the GPT-2-medium projection shapes, in the operand layouts ops/fp8.py keeps
(A [M][K], B [N][K], both K-contiguous), per role: forward e4m3 x e4m3 (+bf16 bias), data gradient e5m2 x e4m3,
weight gradient e5m2 x e4m3 with f32 output; numerics against a dequantized f32 reference; timing next to ours.

    python tools/probe_scaled_mm.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_tensorflow_amd.ops import fp8 as F  # noqa: E402
from tools.bench_kernels import timeit  # noqa: E402

E4, E5, BF = torch.float8_e4m3fn, torch.float8_e5m2, torch.bfloat16


def main():
    dev = torch.device("cuda")
    T = 8192
    torch.manual_seed(0)
    sa = torch.tensor(0.5, device=dev)
    sb = torch.tensor(0.25, device=dev)
    sc2 = torch.stack([sa, sb]).float()
    for name, kin, kout in (("qkv", 1024, 3072), ("out", 1024, 1024), ("ffn1", 1024, 4096), ("ffn2", 4096, 1024)):
        for role in ("fwd", "dX", "dW"):
            if role == "fwd":
                M, N, K, ta, tb = T, kout, kin, E4, E4
            elif role == "dX":
                M, N, K, ta, tb = T, kin, kout, E5, E4
            else:
                M, N, K, ta, tb = kout, kin, T, E5, E4
            a = (torch.randn(M, K, device=dev) * 2).to(ta)
            b = (torch.randn(N, K, device=dev) * 2).to(tb)
            bias = (torch.randn(N, device=dev) * 0.1).to(BF) if role == "fwd" else None
            od = torch.float32 if role == "dW" else BF
            try:
                y = torch._scaled_mm(a, b.t(), scale_a=sa, scale_b=sb, bias=bias, out_dtype=od)
            except Exception as e:  # noqa: BLE001
                print(f"{name} {role}: _scaled_mm failed: {str(e)[:150]}", flush=True)
                continue
            ref = (a.float() * 0.5) @ (b.float() * 0.25).t() + (bias.float() if bias is not None else 0)
            err = (y.float() - ref).abs().max().item() / ref.abs().max().item()
            t = timeit(lambda: torch._scaled_mm(a, b.t(), scale_a=sa, scale_b=sb, bias=bias, out_dtype=od))
            au, bu = a.view(torch.uint8), b.view(torch.uint8)
            out = torch.empty(M, N, dtype=od, device=dev)
            if role == "dW":
                ours = lambda: F.gemm_fp8(au, bu, sc2, out, fmt_a=1, out_f32=True, beta=1.0)
            else:
                ours = lambda: F.gemm_fp8(au, bu, sc2, out, fmt_a=0 if role == "fwd" else 1, bias=None)
            to = timeit(ours)
            fl = 2.0 * M * N * K
            print(f"{name:4s} {role:3s} M={M} N={N} K={K}: hipBLASLt {t * 1e6:6.1f}us {fl / t / 1e12:5.0f} TF "
                  f"(rel err {err:.1e}) | ours {to * 1e6:6.1f}us {fl / to / 1e12:5.0f} TF", flush=True)


if __name__ == "__main__":
    main()
