#!/usr/bin/env python
"""GPT-2-medium fp8: per-parameter gradient difference of the fused FFN epilogue path vs the unfused one (same init,
same batch; step 1 bootstraps the delayed scales, gradients compared on step 2) and of both vs the bf16 model."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_tensorflow_amd.data import synthetic_tokens  # noqa: E402
from distributed_tensorflow_amd.keras import initializers  # noqa: E402
from distributed_tensorflow_amd.models.transformer import GPT2  # noqa: E402
from distributed_tensorflow_amd.ops import fp8  # noqa: E402


def grads(fp8_on, fuse_bwd, layers=4):
    fp8._FUSE_BWD = fuse_bwd
    initializers.set_seed(5)
    dev = torch.device("cuda")
    model = GPT2(hidden=1024, layers=layers, heads=16, dropout=0.0, fp8=fp8_on)
    data = iter(synthetic_tokens(8, 1024, 50257, dev, seed=0))
    out = None
    for _ in range(2):
        x, y = next(data)
        for p in model.trainable_weights:
            p.grad = None
        logits = model(x, training=True)
        loss = torch.nn.functional.cross_entropy(logits.float().reshape(-1, logits.shape[-1])[:, :50257],
                                                 y.reshape(-1))
        loss.backward()
        torch.cuda.synchronize()
        out = {i: (getattr(p, "name", str(i)), p.grad.float().clone()) for i, p in enumerate(model.trainable_weights)
               if p.grad is not None}
    return out


def rel(a, b):
    return ((a - b).norm() / (b.norm() + 1e-20)).item()


f = grads(True, True)
u = grads(True, False)
b = grads(False, True)
for i in sorted(b):
    n = b[i][0]
    print(f"{n:55s} fused-vs-unfused {rel(f[i][1], u[i][1]):.4f}  fused-vs-bf16 {rel(f[i][1], b[i][1]):.4f}  "
          f"unfused-vs-bf16 {rel(u[i][1], b[i][1]):.4f}  |g| f/u {f[i][1].norm().item() / (u[i][1].norm().item() + 1e-20):.4f}")
