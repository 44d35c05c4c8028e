"""The space-to-depth stem's weight gradient (ResNet-50, batch 256: dW [64][4][4][16] over 3.2M output pixels) per
forced tile and split-K, against its MFMA floor. python tools/stem_wgrad_probe.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_tensorflow_amd.ops._util import call, ptr, stream, workspace  # noqa: E402


def timeit(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    dev = torch.device("cuda")
    N, Hs, C, K, R = 256, 115, 16, 64, 4
    P = Hs - R + 1  # 112
    x = (torch.rand(N, Hs, Hs, C, device=dev) * 2 - 1).to(torch.bfloat16)
    dy = (torch.rand(N, P, P, K, device=dev) * 2 - 1).to(torch.bfloat16)
    dw = torch.zeros(K, R, R, C, device=dev)
    ws = workspace(dev)
    fl = 2.0 * N * P * P * K * R * R * C
    print(f"stem s2d wgrad: {fl / 1e9:.0f} GFLOP, floor {fl / 1.3e15 * 1e6:.0f} us at 1.3 PF", flush=True)
    for tile in (-1, 0, 1, 2, 3, 4, 7, 8, 9, 15, 16):
        for sk in (0, 64, 128, 256, 512):
            def run():
                call("dtf_conv_wgrad", ptr(x), ptr(dy), ptr(dw), N, Hs, Hs, C, K, R, R, P, P, 1, 1, 0, 0, 1, 1, 0, sk,
                     tile, ptr(ws), ws.numel(), stream())
            try:
                us = timeit(run)
            except Exception as e:  # noqa: BLE001
                print(f"tile {tile:3d} splitk {sk:4d}: {e}", flush=True)
                continue
            print(f"tile {tile:3d} splitk {sk:4d}: {us:7.1f} us  {fl / us / 1e6:6.0f} TF", flush=True)


if __name__ == "__main__":
    main()
