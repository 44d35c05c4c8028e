"""The 4-wave 256x256 GEMM (csrc/kernels/gemm_w4.hip) against the 8-wave gemm256 kernel and hipBLASLt (torch.mm,
test oracle only) on the transformer / square shapes, in the three layouts the dense layers use:
  NT  forward         A [M][K] x B [N][K]^T        -> bf16
  NN  data gradient   A [M][K] x B [K][N]          -> bf16
  TN  weight gradient A [K][M]^T x B [K][N]        -> f32
Correctness against an f32 product, then TF/s over interleaved rounds in one process (cdna_hip_programming.md §5.4
rule 24) on uniform random [-1, 1) operands (rule 25).

    python tools/bench_gemm_w4.py [--rounds 3] [--shapes 8192x8192x8192,...] [--layouts NT,NN,TN]"""
import argparse
import sys
import time

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from distributed_tensorflow_amd.ops._util import call, ptr, stream, workspace  # noqa: E402

SHAPES = [(4096, 4096, 4096), (8192, 8192, 8192), (16384, 768, 768), (16384, 3072, 768), (16384, 768, 3072),
          (16384, 2304, 768), (8192, 1024, 1024), (8192, 3072, 1024), (8192, 4096, 1024), (8192, 1024, 4096)]


def timeit(fn, iters):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters


def ablate(a):
    """TF/s of the NT kernel and its ablation builds (1 no LDS-DMA, 2 no fragment reads, 3 neither)."""
    dev = torch.device("cuda")
    shapes = [(8192, 8192, 8192), (4096, 4096, 4096), (16384, 3072, 768)] if not a.shapes else [
        tuple(int(v) for v in s.split("x")) for s in a.shapes.split(",")]
    for (M, N, K) in shapes:
        A = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
        B = (torch.rand(N, K, device=dev) * 2 - 1).to(torch.bfloat16)
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        fl = 2.0 * M * N * K
        iters = max(3, min(50, int(2e13 / fl)))
        res = {v: [] for v in range(4)}
        for _ in range(a.rounds):
            for v in range(4):
                res[v].append(timeit(lambda: call("dtf_gemm_w4_var", ptr(A), ptr(B), ptr(out), M, N, K, v, 256,
                                                  stream()), iters))
        print(f"{M}x{N}x{K}: " + "  ".join(f"var{v} {fl / min(r) / 1e12:7.1f} TF" for v, r in res.items()), flush=True)
    return 0


def sweepk(a):
    dev = torch.device("cuda")
    M, N = (int(v) for v in a.sweepk.split("x"))
    for K in (256, 512, 768, 1536, 3072, 6144):
        A = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
        B = (torch.rand(N, K, device=dev) * 2 - 1).to(torch.bfloat16)
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        res = {"w4": [], "noepi": [], "blas": []}
        for _ in range(a.rounds):
            res["w4"].append(timeit(lambda: call("dtf_gemm_w4", ptr(A), ptr(B), ptr(out), M, N, K, K, K, N, 0, 0, 0,
                                                 256, stream()), 20))
            res["noepi"].append(timeit(lambda: call("dtf_gemm_w4_var", ptr(A), ptr(B), ptr(out), M, N, K, 4,
                                                    256, stream()), 20))
            res["blas"].append(timeit(lambda: A @ B.t(), 20))
        print(f"{M}x{N}x{K:5d}: w4 {min(res['w4']) * 1e6:8.1f} us  w4-no-epilogue {min(res['noepi']) * 1e6:8.1f} us  "
              f"hipblaslt {min(res['blas']) * 1e6:8.1f} us", flush=True)
    return 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--shapes", default=None)
    ap.add_argument("--layouts", default="NT,NN,TN")
    ap.add_argument("--var", action="store_true", help="ablation builds of the NT kernel (timing only)")
    ap.add_argument("--sweepk", default=None, help="MxN: time the NT kernel over K (fixed cost vs per-K-tile cost)")
    a = ap.parse_args()
    if a.var:
        return ablate(a)
    if a.sweepk:
        return sweepk(a)
    shapes = SHAPES if not a.shapes else [tuple(int(v) for v in s.split("x")) for s in a.shapes.split(",")]
    dev = torch.device("cuda")
    torch.manual_seed(0)
    ok = True
    ws = workspace(dev)
    for lay in a.layouts.split(","):
        for (M, N, K) in shapes:
            ako, bko = lay[0] == "T", lay[1] == "N"
            A = (torch.rand((K, M) if ako else (M, K), device=dev) * 2 - 1).to(torch.bfloat16)
            B = (torch.rand((K, N) if bko else (N, K), device=dev) * 2 - 1).to(torch.bfloat16)
            f32 = lay == "TN"
            odt = torch.float32 if f32 else torch.bfloat16
            out = torch.empty(M, N, device=dev, dtype=odt)
            o2 = torch.empty_like(out)
            o3 = torch.empty_like(out)
            lda, ldb = A.stride(0), B.stride(0)

            def w4():
                call("dtf_gemm_w4", ptr(A), ptr(B), ptr(out), M, N, K, lda, ldb, N, int(ako), int(bko), int(f32),
                     256, stream())

            def w4n():
                call("dtf_gemm_w4", ptr(A), ptr(B), ptr(o3), M, N, K, lda, ldb, N, int(ako), int(bko), int(f32),
                     128, stream())

            def g256():
                call("dtf_gemm256", ptr(A), ptr(B), ptr(o2), M, N, K, lda, ldb, N, int(ako), int(bko), int(f32), 1,
                     ptr(ws), ws.numel(), stream())

            At = A.t() if ako else A
            Bt = B if bko else B.t()

            def blas():
                if f32:
                    return torch.mm(At, Bt, out_dtype=torch.float32)
                return torch.mm(At, Bt)

            w4()
            w4n()
            torch.cuda.synchronize()
            ref = At.float() @ Bt.float()
            err = max((o.float() - ref).abs().max().item() for o in (out, o3)) / (ref.abs().max().item() + 1e-6)
            good = err < 1e-2
            ok &= good
            fl = 2.0 * M * N * K
            iters = max(3, min(50, int(2e13 / fl)))
            res = {"w4": [], "w4n": [], "g256": [], "blas": []}
            for _ in range(a.rounds):
                res["w4"].append(timeit(w4, iters))
                res["w4n"].append(timeit(w4n, iters))
                res["g256"].append(timeit(g256, iters))
                res["blas"].append(timeit(blas, iters))
            tf = {k: fl / min(v) / 1e12 for k, v in res.items()}
            print(f"{lay} {M:6d}x{N:5d}x{K:5d} err={err:.1e} {'OK ' if good else 'BAD'}  w4 {tf['w4']:7.1f} TF  w4n {tf['w4n']:7.1f} TF  "
                  f"g256 {tf['g256']:7.1f} TF  hipblaslt {tf['blas']:7.1f} TF  (best/blas {max(tf['w4'], tf['w4n']) / tf['blas']:.2f}, "
                  f"w4/g256 {tf['w4'] / tf['g256']:.2f})", flush=True)
    print("ALL OK" if ok else "FAILURES")
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
