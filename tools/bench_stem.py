"""Stem convolution variants (ResNet-50, batch 256): the 7x7/2 conv over 8-channel-padded NHWC images vs the
same conv as a 4x4/1 conv over the 2x2 space-to-depth image [N, 115, 115, 16] (3 colour channels padded to 4,
2/1 rows of zero padding baked in). Times forward (with BN statistics) and weight gradient per tile.

  python tools/bench_stem.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_tensorflow_amd.ops import conv as C  # noqa: E402
from distributed_tensorflow_amd.ops._util import IntOut, call, ptr, stream, workspace  # noqa: E402
from tools.conv_roofline import timeit  # noqa: E402

BF = torch.bfloat16
NB = 256


def run(name, H, Cin, R, s, p):
    dev = torch.device("cuda")
    x = torch.randn(NB, H, H, Cin, device=dev).to(BF)
    w = torch.randn(64, R, R, Cin, device=dev) * 0.05
    w16 = w.to(BF)
    g = C._geom(x, w, (s, s), (p, p), (1, 1))
    P, Q = g[7], g[8]
    dy = torch.randn(NB, P, Q, 64, device=dev).to(BF)
    M = NB * P * Q
    ws = workspace(dev)
    dwacc = torch.zeros(64, R, R, Cin, device=dev)
    part = torch.empty(((M + 63) // 64) * 2 * 64, dtype=torch.float32, device=dev)
    rows = IntOut()
    y = torch.empty(NB, P, Q, 64, device=dev, dtype=BF)
    fl = 2.0 * M * 64 * R * R * Cin
    for kind in ("fwd", "wgrad"):
        line = f"{name:10s} {kind:5s} P={P} K={R * R * Cin}"
        for tile in [-1] + list(range(0, 11)):
            if kind == "fwd":
                fn = lambda t=tile: call("dtf_conv_fwd", ptr(x), ptr(w16), ptr(y), None, ptr(part), rows.addr, NB, H,
                                         H, Cin, 64, R, R, P, Q, s, s, p, p, 1, 1, 0, 0, t, stream())
            else:
                fn = lambda t=tile: call("dtf_conv_wgrad", ptr(x), ptr(dy), ptr(dwacc), NB, H, H, Cin, 64, R, R, P, Q,
                                         s, s, p, p, 1, 1, 1, 0, t, ptr(ws), ws.numel(), stream())
            try:
                tt = timeit(fn)
            except Exception:  # noqa: BLE001 - tile not instantiated for this operand mode
                continue
            line += f" t{tile}:{tt * 1e6:.0f}us({fl / tt / 1e12:.0f}TF)"
        print(line, flush=True)


if __name__ == "__main__":
    torch.manual_seed(0)
    run("stem7x7", 224, 8, 7, 2, 3)
    run("stem_s2d", 115, 16, 4, 1, 0)
