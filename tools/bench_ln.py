#!/usr/bin/env python
"""Bandwidth of the LayerNorm kernels at the BERT-base (16384 x 768) and GPT-2-medium (8192 x 1024) shapes, alone
on the GPU (in a training step they share CUs with the weight-gradient GEMMs of the side stream).

    python tools/bench_ln.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_tensorflow_amd.ops._util import call, ptr, stream  # noqa: E402
from tools.bench_kernels import timeit  # noqa: E402

BF = torch.bfloat16


def main():
    dev = torch.device("cuda")
    for M, D in [(16384, 768), (8192, 1024), (16384, 1024)]:
        x = torch.randn(M, D, device=dev).to(BF)
        dy = torch.randn(M, D, device=dev).to(BF)
        y = torch.empty_like(x)
        dx = torch.empty_like(x)
        g = torch.rand(D, device=dev) + 0.5
        b = torch.randn(D, device=dev)
        mean = torch.empty(M, device=dev)
        rstd = torch.empty(M, device=dev)
        dgb = torch.zeros(2 * D, device=dev)
        ws = torch.empty(1024 * 2 * D + 16, device=dev)
        n = M * D * 2
        t_copy = timeit(lambda: y.copy_(x))
        t_f = timeit(lambda: call("dtf_layernorm_fwd", ptr(x), ptr(g), ptr(b), ptr(y), ptr(mean), ptr(rstd), M, D,
                                  1e-5, stream()))
        t_b = timeit(lambda: call("dtf_layernorm_bwd", ptr(dy), ptr(x), ptr(g), ptr(mean), ptr(rstd), ptr(dx),
                                  ptr(dgb), ptr(ws), ws.numel(), M, D, 0, stream()))
        xf = x.float().requires_grad_()
        ref = torch.nn.functional.layer_norm(xf, (D,), g, b, 1e-5)
        ref.backward(dy.float())
        err = float((dx.float() - xf.grad).abs().max() / xf.grad.abs().max())
        gb = lambda nb, t: nb / t / 1e9  # noqa: E731
        print(f"M={M:6d} D={D:5d} copy {gb(2 * n, t_copy):6.0f} GB/s | fwd {t_f * 1e6:6.1f}us {gb(2 * n, t_f):6.0f} GB/s"
              f" | bwd {t_b * 1e6:6.1f}us {gb(3 * n, t_b):6.0f} GB/s (dx rel err {err:.1e})", flush=True)


if __name__ == "__main__":
    main()
