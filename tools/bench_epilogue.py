#!/usr/bin/env python
"""Cost of the GEMM epilogue pieces on the FFN1 shapes (ops.linalg.gemm, bf16): plain, +bias, +GELU, +pre-activation
side output (aux), +both — python tools/bench_epilogue.py"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_tensorflow_amd.ops.linalg import gemm  # noqa: E402

dev = torch.device("cuda")
for name, M, K, N in (("bert ffn1", 16384, 768, 3072), ("gpt2 ffn1", 8192, 1024, 4096)):
    x = torch.randn(M, K, device=dev).to(torch.bfloat16)
    w = (torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)
    b = torch.zeros(N, device=dev)
    aux = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    for label, kw in (("plain", {}), ("bias", dict(bias=b)), ("bias+gelu", dict(bias=b, act=2)),
                      ("bias+aux", dict(bias=b, aux=aux)), ("bias+gelu+aux", dict(bias=b, act=2, aux=aux))):
        for _ in range(3):
            gemm(x, w, **kw)
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(20):
            gemm(x, w, **kw)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t) / 20
        print(f"{name} {label:14s} {dt * 1e6:7.1f} us  {2 * M * N * K / dt / 1e12:6.0f} TF", flush=True)
