"""The 8-phase 256x256 kernel (csrc/kernels/gemm8p.hip) vs the 4-phase gemm256 kernel and hipBLASLt (torch.matmul)
on NT GEMMs (A [M][K], B [N][K]): correctness against an f32 product and TF/s, interleaved rounds in one process
(cdna_hip_programming.md §5.4 rule 24), uniform random [-1, 1) operands (rule 25).

    python tools/bench_gemm8p.py [--rounds 3] [--shapes 8192x8192x8192,...]"""
import argparse
import sys
import time

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from distributed_tensorflow_amd.ops._util import call, ptr, stream, workspace  # noqa: E402

SHAPES = [(4096, 4096, 4096), (8192, 8192, 8192), (16384, 3072, 768), (16384, 768, 3072), (16384, 2304, 768),
          (8192, 4096, 1024), (8192, 1024, 4096), (50176, 256, 2304), (12544, 512, 4608), (200704, 128, 1152)]


def timeit(fn, iters):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--shapes", default=None)
    a = ap.parse_args()
    shapes = SHAPES if not a.shapes else [tuple(int(v) for v in s.split("x")) for s in a.shapes.split(",")]
    dev = torch.device("cuda")
    torch.manual_seed(0)
    ok = True
    for (M, N, K) in shapes:
        A = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
        B = (torch.rand(N, K, device=dev) * 2 - 1).to(torch.bfloat16)
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        o2 = torch.empty_like(out)
        ws = workspace(dev)

        o3 = torch.empty_like(out)

        def k8():
            call("dtf_gemm8p", ptr(A), ptr(B), ptr(out), M, N, K, K, K, N, 0, 256, stream())

        def k8n():
            call("dtf_gemm8p", ptr(A), ptr(B), ptr(o3), M, N, K, K, K, N, 0, 128, stream())

        def k256():
            call("dtf_gemm256", ptr(A), ptr(B), ptr(o2), M, N, K, K, K, N, 0, 0, 0, 1, ptr(ws), ws.numel(), stream())

        def blas():
            return A @ B.t()

        k8()
        k8n()
        torch.cuda.synchronize()
        ref = A.float() @ B.float().t()
        err = (out.float() - ref).abs().max().item() / (ref.abs().max().item() + 1e-6)
        err = max(err, (o3.float() - ref).abs().max().item() / (ref.abs().max().item() + 1e-6))
        good = err < 1e-2
        ok &= good
        fl = 2.0 * M * N * K
        iters = max(3, min(50, int(2e13 / fl)))
        res = {"8p": [], "8p128": [], "g256": [], "blas": []}
        for _ in range(a.rounds):
            res["8p"].append(timeit(k8, iters))
            res["8p128"].append(timeit(k8n, iters))
            res["g256"].append(timeit(k256, iters))
            res["blas"].append(timeit(blas, iters))
        tf = {k: fl / min(v) / 1e12 for k, v in res.items()}
        print(f"{M:6d}x{N:5d}x{K:5d} err={err:.1e} {'OK ' if good else 'BAD'}  8p {tf['8p']:7.1f} TF  "
              f"8p128 {tf['8p128']:7.1f} TF  g256 {tf['g256']:7.1f} TF  hipblaslt {tf['blas']:7.1f} TF  (8p/g256 {tf['8p'] / tf['g256']:.2f}, "
              f"8p/blas {tf['8p'] / tf['blas']:.2f})", flush=True)
    print("ALL OK" if ok else "FAILURES")
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
