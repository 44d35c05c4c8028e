#!/usr/bin/env python
"""Bandwidth of the channels-last BatchNorm passes at the ResNet-50 (batch 256) shapes vs a torch copy.

    python tools/bench_bn.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_tensorflow_amd.ops._util import call, ptr, stream  # noqa: E402
from tools.bench_kernels import timeit  # noqa: E402

BF = torch.bfloat16
SHAPES = [(3211264, 64), (802816, 64), (802816, 256), (200704, 128), (200704, 512), (50176, 256), (50176, 1024),
          (12544, 512), (12544, 2048)]


def main():
    dev = torch.device("cuda")
    for M, C in SHAPES:
        x = torch.randn(M, C, device=dev).to(BF)
        dy = torch.randn(M, C, device=dev).to(BF)
        res = torch.randn(M, C, device=dev).to(BF)
        y = torch.empty_like(x)
        dx = torch.empty_like(x)
        dz = torch.empty_like(x)
        mb = torch.empty(M * C // 8, dtype=torch.uint8, device=dev)
        sc = torch.rand(C, device=dev) + 0.5
        sh = torch.randn(C, device=dev)
        mean = torch.randn(C, device=dev) * 0.1
        inv = torch.rand(C, device=dev) + 0.5
        gm = torch.rand(C, device=dev) + 0.5
        dg = torch.zeros(C, device=dev)
        db = torch.zeros(C, device=dev)
        work = torch.empty((2 * 1024 + 3) * C, device=dev)
        n = M * C * 2  # bytes of one bf16 tensor
        t_copy = timeit(lambda: y.copy_(x))
        t_app = timeit(lambda: call("dtf_bn_apply", ptr(x), ptr(sc), ptr(sh), None, ptr(y), M, C, 1, ptr(mb), None, None,
                                    stream()))
        t_res = timeit(lambda: call("dtf_bn_apply", ptr(x), ptr(sc), ptr(sh), ptr(res), ptr(y), M, C, 1, ptr(mb), None, None,
                                    stream()))
        t_bwd = timeit(lambda: call("dtf_bn_bwd", ptr(dy), None, ptr(mb), ptr(x), ptr(mean), ptr(inv), ptr(gm), M, C,
                                    ptr(dx), None, ptr(dg), ptr(db), 0, ptr(work), None, None, None, None, None, None, stream()))
        t_bwdr = timeit(lambda: call("dtf_bn_bwd", ptr(dy), None, ptr(mb), ptr(x), ptr(mean), ptr(inv), ptr(gm), M,
                                     C, ptr(dx), ptr(dz), ptr(dg), ptr(db), 0, ptr(work), None, None, None, None, None, None, stream()))
        rows = max(1, M // 128)
        part = torch.randn(rows, 2 * C, device=dev) * 0.01
        coef = torch.empty(3 * C, device=dev)
        # the apply-only backward the model runs when the consumer's dgrad epilogue already reduced (bn_bwd_apply)
        t_bp = timeit(lambda: call("dtf_bn_bwd_partials", ptr(dy), ptr(mb), ptr(x), ptr(mean), ptr(inv), ptr(gm), M, C,
                                   ptr(dx), None, ptr(dg), ptr(db), 0, ptr(part), rows, ptr(coef), None, None, None,
                                   None, stream()))
        t_bpr = timeit(lambda: call("dtf_bn_bwd_partials", ptr(dy), ptr(mb), ptr(x), ptr(mean), ptr(inv), ptr(gm), M,
                                    C, ptr(dx), ptr(dz), ptr(dg), ptr(db), 0, ptr(part), rows, ptr(coef), None, None,
                                    None, None, stream()))
        gb = lambda b, t: b / t / 1e9  # noqa: E731
        print(f"M={M:8d} C={C:5d} bwd apply-only {t_bp * 1e6:7.1f}us {gb(3.0625 * n, t_bp):6.0f} GB/s | "
              f"+dres {t_bpr * 1e6:7.1f}us {gb(4.0625 * n, t_bpr):6.0f} GB/s", flush=True)
        print(f"M={M:8d} C={C:5d} copy {gb(2 * n, t_copy):6.0f} GB/s | apply {t_app * 1e6:7.1f}us "
              f"{gb(2.0625 * n, t_app):6.0f} GB/s | apply+res {t_res * 1e6:7.1f}us {gb(3.0625 * n, t_res):6.0f} | "
              f"bwd {t_bwd * 1e6:7.1f}us {gb(5.125 * n, t_bwd):6.0f} | bwd+dz {t_bwdr * 1e6:7.1f}us "
              f"{gb(6.125 * n, t_bwdr):6.0f}", flush=True)


if __name__ == "__main__":
    main()
