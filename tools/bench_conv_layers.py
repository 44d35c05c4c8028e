"""Per-layer timing of ResNet-50's 1x1 convolutions (batch 256) through our kernels: fwd with/without the
BN-statistics epilogue and each tile shape, vs the memory floor (bytes moved at 5 TB/s)."""
import sys
import time

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from distributed_tensorflow_amd.ops import conv as C  # noqa: E402
from distributed_tensorflow_amd.ops._util import IntOut, call, ptr, stream  # noqa: E402


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters


dev = torch.device("cuda")
for (HW, Cin, K) in [(56, 64, 256), (56, 256, 64), (56, 64, 64), (28, 128, 512), (28, 512, 128), (14, 256, 1024),
                     (14, 1024, 256), (7, 512, 2048), (7, 2048, 512)]:
    N = 256
    x = torch.randn(N, HW, HW, Cin, device=dev).to(torch.bfloat16)
    w = (torch.randn(K, 1, 1, Cin, device=dev) * 0.05).to(torch.bfloat16)
    y = torch.empty(N, HW, HW, K, device=dev, dtype=torch.bfloat16)
    M = N * HW * HW
    part = torch.empty(((M + 63) // 64) * 2 * K, dtype=torch.float32, device=dev)
    rows = IntOut()
    res = []
    for stats in (0, 1):
        for tile in (-1, 0, 1, 2):
            def f():
                call("dtf_conv_fwd", ptr(x), ptr(w), ptr(y), None, ptr(part) if stats else None,
                     rows.addr if stats else None, N, HW, HW, Cin, K, 1, 1, HW, HW, 1, 1, 0, 0, 1, 1, 0, 0, tile,
                     stream())
            res.append((stats, tile, timeit(f)))
    fl = 2.0 * M * Cin * K
    floor = (M * Cin + M * K) * 2 / 5e12
    s = "  ".join(f"s{st}t{tl}:{t * 1e3:.3f}ms({fl / t / 1e12:.0f}TF)" for st, tl, t in res)
    print(f"M={M} C={Cin} K={K} floor={floor * 1e3:.3f}ms  {s}", flush=True)
