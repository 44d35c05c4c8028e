#!/usr/bin/env python
"""Latency of the BatchNorm partial-row reduce + finalize launch (dtf_bn_finalize) at the ResNet-50 b256 shapes:
T partial rows (one per 128-row GEMM tile) x 2C floats.

    python tools/bench_bn_finalize.py            (DTF_BN_GROUPS=<n> caps the group count)
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_tensorflow_amd.ops._util import call, ptr, stream  # noqa: E402
from tools.bench_kernels import timeit  # noqa: E402

SHAPES = [(6272, 64), (6272, 256), (1568, 128), (1568, 512), (392, 256), (392, 1024), (98, 512), (98, 2048)]


def main():
    dev = torch.device("cuda")
    for T, C in SHAPES:
        part = torch.randn(T * 2 * C, device=dev).abs()
        g = torch.ones(C, device=dev)
        b = torch.zeros(C, device=dev)
        rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
        out = torch.empty(4, C, device=dev)
        t = timeit(lambda: call("dtf_bn_finalize", ptr(part), T, ptr(g), ptr(b), ptr(rm), ptr(rv), T * 128, C, 0.9,
                                1e-5, ptr(out[0]), ptr(out[1]), ptr(out[2]), ptr(out[3]), stream()))
        ref = part.view(T, 2 * C).double().sum(0)
        mean = ref[:C] / (T * 128)
        err = (out[2].double() - mean).abs().max().item() / mean.abs().max().item()
        print(f"T={T:5d} C={C:5d} {t * 1e6:7.1f} us  rel.err(mean) {err:.1e}", flush=True)


if __name__ == "__main__":
    main()
