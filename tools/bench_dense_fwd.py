#!/usr/bin/env python
"""Forward Dense GEMM (ops.dense, bias, optional GELU) timing on the BERT-base / GPT-2-medium projection shapes, as
the model calls it (env knobs of the GEMM dispatch apply): python tools/bench_dense_fwd.py"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_tensorflow_amd import ops  # noqa: E402

dev = torch.device("cuda")
SHAPES = [("bert qkv", 16384, 768, 2304, None), ("bert out", 16384, 768, 768, None),
          ("bert ffn1", 16384, 768, 3072, "gelu"), ("bert ffn2", 16384, 3072, 768, None),
          ("gpt2 qkv", 8192, 1024, 3072, None), ("gpt2 out", 8192, 1024, 1024, None),
          ("gpt2 ffn1", 8192, 1024, 4096, "gelu"), ("gpt2 ffn2", 8192, 4096, 1024, None),
          ("bert ffn1 noact", 16384, 768, 3072, None), ("gpt2 ffn1 noact", 8192, 1024, 4096, None)]
tot = 0.0
for name, M, K, N, act in SHAPES:
    x = torch.randn(M, K, device=dev).to(torch.bfloat16)
    w = torch.randn(N, K, device=dev) * 0.02
    b = torch.zeros(N, device=dev)
    with torch.no_grad():
        for _ in range(3):
            ops.dense(x, w, b, act=act)
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(20):
            ops.dense(x, w, b, act=act)
        torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / 20
    tot += dt
    print(f"{name:16s} {M}x{K}->{N}: {dt * 1e6:7.1f} us  {2 * M * N * K / dt / 1e12:6.0f} TF", flush=True)
print(f"total {tot * 1e6:.1f} us")
