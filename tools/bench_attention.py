"""Fused attention fwd / bwd timing on the BERT-base and GPT-2-medium shapes, with and without attention
dropout (the kernels regenerate the dropout mask from a counter hash in every pass).

  python tools/bench_attention.py
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_tensorflow_amd import ops  # noqa: E402


def timeit(fn, iters=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters


dev = torch.device("cuda")
for name, B, S, H, causal in (("bert", 32, 512, 12, False), ("gpt2", 8, 1024, 16, True)):
    qkv = (torch.randn(B, S, 3 * H * 64, device=dev) * 0.5).to(torch.bfloat16).requires_grad_(True)
    g = torch.randn(B, S, H * 64, device=dev).to(torch.bfloat16)
    fl = 4.0 * B * H * S * S * 64 * (0.5 if causal else 1.0)
    for rate in (0.0, 0.1):
        f = lambda: ops.attention_packed(qkv, H, causal=causal, dropout=rate, training=True, seed=1)
        tf = timeit(lambda: f())
        y = f()
        tb = timeit(lambda: torch.autograd.grad(f(), [qkv], g)) - tf
        print(f"{name} dropout={rate}: fwd {tf * 1e6:7.1f}us ({fl / tf / 1e12:5.0f} TF)  bwd {tb * 1e6:7.1f}us "
              f"({2.5 * fl / tb / 1e12:5.0f} TF)", flush=True)
