#!/usr/bin/env python
"""BatchNorm backward APPLY pass (dx = a*dz + b*x + c with the 1-bit ReLU mask; dtf_bn_bwd_apply_coef) at the
ResNet-50 b256 shapes, for every streaming variant of norm.hip (dtf_set_ew_variant: rows per trip, nontemporal
hints), against a torch copy of the same tensor.

    python tools/bench_bnb.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_tensorflow_amd.ops._util import call, ptr, stream  # noqa: E402
from tools.bench_kernels import timeit  # noqa: E402

BF = torch.bfloat16
SHAPES = [(802816, 64), (802816, 256), (200704, 128), (200704, 512), (50176, 256), (50176, 1024), (12544, 2048)]
VARIANTS = {0: "EU4", 1: "EU4+nt", 2: "EU8", 3: "EU8+nt", 4: "EU2"}


def main():
    dev = torch.device("cuda")
    for M, C in SHAPES:
        x = torch.randn(M, C, device=dev).to(BF)
        dy = torch.randn(M, C, device=dev).to(BF)
        dx = torch.empty_like(x)
        y = torch.empty_like(x)
        mb = torch.randint(0, 256, (M * C // 8,), dtype=torch.uint8, device=dev)
        coef = torch.randn(3 * C, device=dev)
        n = M * C * 2
        t_copy = timeit(lambda: y.copy_(x))
        line = f"M={M:7d} C={C:5d} copy {2 * n / t_copy / 1e9:6.0f} GB/s |"
        for v, nm in VARIANTS.items():
            call("dtf_set_ew_variant", v)
            t = timeit(lambda: call("dtf_bn_bwd_apply_coef", ptr(dy), ptr(mb), ptr(x), M, C, ptr(dx), None, ptr(coef),
                                    None, None, None, None, None, None, stream()))
            line += f" {nm} {t * 1e6:6.1f}us {3.0625 * n / t / 1e9:5.0f}"
        call("dtf_set_ew_variant", 4)
        sc, sh = torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev)
        res = torch.randn(M, C, device=dev).to(BF)
        for nu in (2, 4, 8):
            call("dtf_set_ew_apply_nu", nu)
            t = timeit(lambda: call("dtf_bn_apply", ptr(x), ptr(sc), ptr(sh), ptr(res), ptr(y), M, C, 1, ptr(mb), None,
                                    None, stream()))
            line += f" | apply+res NU{nu} {t * 1e6:6.1f}us {3.0625 * n / t / 1e9:5.0f}"
        call("dtf_set_ew_apply_nu", 2)
        print(line, flush=True)


if __name__ == "__main__":
    main()
