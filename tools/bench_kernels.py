"""Micro-benchmarks of the hand-written gfx950 kernels vs the vendor libraries
(hipBLASLt via torch.matmul, MIOpen via torch conv2d) on the same random data.

  python tools/bench_kernels.py [--quick]
Prints one line per shape: our TFLOP/s, vendor TFLOP/s, ratio.
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_tensorflow_amd import ops  # noqa: E402
from distributed_tensorflow_amd.ops import conv as C  # noqa: E402

BF = torch.bfloat16


def timeit(fn, iters=20, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    s = torch.cuda.Event(enable_timing=True)
    e = torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e-3


def gemm_suite(quick):
    shapes = [(4096, 4096, 4096), (8192, 8192, 8192), (16384, 768, 768), (16384, 3072, 768), (16384, 768, 3072),
              (16384, 2304, 768), (8192, 1024, 4096)]
    if quick:
        shapes = shapes[:3]
    for M, N, K in shapes:
        a = torch.randn(M, K, device="cuda").to(BF)
        b = torch.randn(N, K, device="cuda").to(BF)
        fl = 2.0 * M * N * K
        t_ours = timeit(lambda: ops.gemm(a, b))
        t_ref = timeit(lambda: a @ b.t())
        bt = b.t().contiguous()
        t_nn = timeit(lambda: ops.gemm(a, bt, b_kouter=True))
        at = a.t().contiguous()
        t_tn = timeit(lambda: ops.gemm(at, bt, a_kouter=True, b_kouter=True, out_dtype=torch.float32))
        print(f"GEMM {M}x{N}x{K}: NT {fl / t_ours / 1e12:7.1f} TF | NN {fl / t_nn / 1e12:7.1f} | "
              f"TN {fl / t_tn / 1e12:7.1f} | hipBLASLt {fl / t_ref / 1e12:7.1f} TF  ratio {t_ref / t_ours:.2f}",
              flush=True)


RESNET = [  # N,H,W,C,K,R,S,stride,pad  (batch 256 ResNet-50 v1.5 layer shapes)
    (256, 224, 224, 8, 64, 7, 7, 2, 3),
    (256, 56, 56, 64, 64, 1, 1, 1, 0),
    (256, 56, 56, 64, 64, 3, 3, 1, 1),
    (256, 56, 56, 64, 256, 1, 1, 1, 0),
    (256, 56, 56, 256, 64, 1, 1, 1, 0),
    (256, 56, 56, 128, 128, 3, 3, 2, 1),
    (256, 28, 28, 128, 512, 1, 1, 1, 0),
    (256, 28, 28, 128, 128, 3, 3, 1, 1),
    (256, 14, 14, 256, 256, 3, 3, 1, 1),
    (256, 14, 14, 1024, 256, 1, 1, 1, 0),
    (256, 7, 7, 512, 512, 3, 3, 1, 1),
    (256, 7, 7, 512, 2048, 1, 1, 1, 0),
    (256, 56, 56, 256, 512, 1, 1, 2, 0),
]


def conv_suite(quick):
    rows = RESNET[:4] if quick else RESNET
    tot_ours = tot_ref = 0.0
    for (N, H, W, Cin, K, R, S, st, pd) in rows:
        x = torch.randn(N, H, W, Cin, device="cuda").to(BF)
        w = torch.randn(K, R, S, Cin, device="cuda") * 0.05
        g = C._geom(x, w, (st, st), (pd, pd), (1, 1))
        P, Q = g[7], g[8]
        fl = 2.0 * N * P * Q * K * R * S * Cin
        w16 = w.to(BF)
        t_f = timeit(lambda: C.conv_fwd_raw(x, w16, g), iters=10)
        dy = torch.randn(N, P, Q, K, device="cuda").to(BF)
        t_d = timeit(lambda: C.conv_dgrad_raw(dy, w, g), iters=10) if Cin != 8 else 0.0
        t_w = timeit(lambda: C.conv_wgrad_raw(x, dy, g), iters=10)
        # MIOpen reference (channels_last bf16)
        xr = x.permute(0, 3, 1, 2)
        wr = w16.permute(0, 3, 1, 2)
        t_rf = timeit(lambda: torch.nn.functional.conv2d(xr, wr, stride=st, padding=pd), iters=10)
        xg = xr.detach().requires_grad_(True)
        wg = wr.detach().requires_grad_(True)
        yr = torch.nn.functional.conv2d(xg, wg, stride=st, padding=pd)
        dyr = dy.permute(0, 3, 1, 2)

        def ref_bwd():
            torch.autograd.grad(yr, [xg, wg] if Cin != 8 else [wg], dyr, retain_graph=True)
        t_rb = timeit(ref_bwd, iters=10)
        ours = t_f + t_d + t_w
        tot_ours += ours
        tot_ref += t_rf + t_rb
        print(f"CONV N{N} {H}x{W} C{Cin}->K{K} {R}x{S}/s{st}: fwd {fl / t_f / 1e12:6.1f} TF "
              f"dgrad {(fl / t_d / 1e12) if t_d else 0:6.1f} wgrad {fl / t_w / 1e12:6.1f} | "
              f"ours {ours * 1e3:7.2f} ms  MIOpen fwd+bwd {(t_rf + t_rb) * 1e3:7.2f} ms", flush=True)
    print(f"CONV total ours {tot_ours * 1e3:.1f} ms vs MIOpen {tot_ref * 1e3:.1f} ms")


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--quick", action="store_true")
    ap.add_argument("--only", default="gemm,conv")
    a = ap.parse_args()
    torch.manual_seed(0)
    print(torch.cuda.get_device_name(0))
    if "gemm" in a.only:
        gemm_suite(a.quick)
    if "conv" in a.only:
        conv_suite(a.quick)
