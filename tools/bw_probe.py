"""Why the channel-expanding pointwise convolutions (ResNet-50 c3 / projection forward: output 4x the input) run
below the HBM roofline: per layer shape, the write-only and copy bandwidth of the output-sized tensor, our 1x1 conv
forward with and without the BN-statistics epilogue (default and forced tiles), and hipBLASLt on the same product.

    python tools/bw_probe.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_tensorflow_amd.ops._util import IntOut, call, ptr, stream  # noqa: E402

BF = torch.bfloat16
SHAPES = [("s1.c3", 802816, 64, 256), ("s2.c3", 200704, 128, 512), ("s3.c3", 50176, 256, 1024),
          ("s4.c3", 12544, 512, 2048), ("s3.c1", 50176, 1024, 256), ("s1.c1", 802816, 256, 64)]


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


def main():
    dev = torch.device("cuda")
    torch.manual_seed(0)
    big = torch.empty(1 << 28, dtype=BF, device=dev)  # 512 MiB: flushes the 256 MB MALL between probes
    for name, M, Cin, K in SHAPES:
        x = torch.randn(M, Cin, device=dev).to(BF)
        w = (torch.randn(K, Cin, device=dev) * 0.05).to(BF)
        y = torch.empty(M, K, device=dev, dtype=BF)
        y2 = torch.empty_like(y)
        part = torch.empty(((M + 63) // 64) * 2 * K, dtype=torch.float32, device=dev)
        rows = IntOut()
        ob, ib = y.numel() * 2, x.numel() * 2
        res = {}
        res["fill"] = timeit(lambda: y.fill_(1.0))
        res["copy"] = timeit(lambda: y2.copy_(y))

        def conv(stats, tile):
            return lambda: call("dtf_conv_fwd", ptr(x), ptr(w), ptr(y), None, ptr(part) if stats else None,
                                rows.addr, 1, M, 1, Cin, K, 1, 1, M, 1, 1, 1, 0, 0, 1, 1, 0, 0, tile, stream())
        res["conv+st"] = timeit(conv(True, -1))
        res["conv"] = timeit(conv(False, -1))
        for t in (0, 2, 7, 8, 9):
            try:
                res[f"t{t}+st"] = timeit(conv(True, t))
            except Exception:  # noqa: BLE001
                pass
        wt = w.t().contiguous()
        res["blas"] = timeit(lambda: torch.matmul(x, wt, out=y2))
        big.fill_(0)
        line = f"{name:6s} M={M:6d} Cin={Cin:4d} K={K:4d} out={ob / 1e6:6.1f}MB in={ib / 1e6:6.1f}MB |"
        line += f" fill {ob / res['fill'] / 1e12:4.2f}TB/s copy {2 * ob / res['copy'] / 1e12:4.2f}TB/s |"
        for k, v in res.items():
            if k in ("fill", "copy"):
                continue
            line += f" {k} {v * 1e6:6.1f}us ({(ob + ib) / v / 1e12:4.2f}TB/s)"
        print(line, flush=True)


if __name__ == "__main__":
    main()
