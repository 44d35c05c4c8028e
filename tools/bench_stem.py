"""Stem convolution variants (ResNet-50, batch 256): the 7x7/2 conv over 8-channel-padded NHWC images vs the
same conv as a 4x4/1 conv over the 2x2 space-to-depth image [N, 115, 115, 16] (3 colour channels padded to 4,
2/1 rows of zero padding baked in). Times forward (with BN statistics) and weight gradient per tile.

  python tools/bench_stem.py
  python tools/bench_stem.py --wgrad-s2d [BATCH]   # s2d weight gradient: persistent stem kernel vs the general tiles
  python tools/bench_stem.py --wgrad-3x3 [BATCH]   # stage-1 3x3 (64 -> 64, 56 x 56) weight gradient, c3wgrad.hip vs tiles
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


def wgrad_s2d(nb):
    dev = torch.device("cuda")
    x = torch.randn(nb, 115, 115, 16, device=dev).to(BF)
    dy = torch.randn(nb, 112, 112, 64, device=dev).to(BF)
    g = (nb, 115, 115, 16, 64, 4, 4, 112, 112, 1, 1, 0, 0, 1, 1)
    ws = workspace(dev)
    dw = torch.zeros(64, 4, 4, 16, device=dev)
    fl = 2.0 * nb * 112 * 112 * 64 * 256
    gb = (x.numel() + dy.numel()) * 2 / 1e9
    stem = lambda: call("dtf_stem_wgrad", ptr(x), ptr(dy), ptr(dw), nb, 115, 115, 0, ptr(ws), ws.numel(), stream())
    gen = lambda: call("dtf_conv_wgrad", ptr(x), ptr(dy), ptr(dw), nb, 115, 115, 16, 64, 4, 4, 112, 112, 1, 1, 0, 0,
                       1, 1, 0, 0, -1, ptr(ws), ws.numel(), stream())
    for name, fn in (("stem kernel", stem), ("general", gen), ("stem kernel", stem)):
        tt = timeit(fn)
        print(f"s2d wgrad batch {nb} {name:12s} {tt * 1e6:8.1f}us  {fl / tt / 1e12:5.0f} TF  {gb / tt / 1e3:5.2f} TB/s "
              f"(x + dY = {gb:.2f} GB)", flush=True)
    a = C.stem_wgrad_raw(x, dy, g)
    b = C.conv_wgrad_raw(x, dy, g)
    print(f"max |stem - general| = {(a - b).abs().max().item():.3e} (max |dW| {b.abs().max().item():.3e})")


def wgrad_3x3(nb):
    dev = torch.device("cuda")
    x = torch.randn(nb, 56, 56, 64, device=dev).to(BF)
    dy = torch.randn(nb, 56, 56, 64, device=dev).to(BF)
    ws = workspace(dev)
    dw = torch.zeros(64, 3, 3, 64, device=dev)
    fl = 2.0 * nb * 56 * 56 * 64 * 576
    gb = (x.numel() + dy.numel()) * 2 / 1e9
    run = lambda: call("dtf_conv_wgrad", ptr(x), ptr(dy), ptr(dw), nb, 56, 56, 64, 64, 3, 3, 56, 56, 1, 1, 1, 1, 1, 1,
                       0, 0, -1, ptr(ws), ws.numel(), stream())
    for on in (1, 0, 1):
        call("dtf_set_c3_wgrad", on)
        tt = timeit(run)
        print(f"3x3 wgrad batch {nb} {'c3wgrad' if on else 'general':8s} {tt * 1e6:8.1f}us  {fl / tt / 1e12:5.0f} TF  "
              f"{gb / tt / 1e3:5.2f} TB/s", flush=True)
    call("dtf_set_c3_wgrad", 1)


if __name__ == "__main__":
    torch.manual_seed(0)
    if len(sys.argv) > 1 and sys.argv[1] == "--wgrad-3x3":
        wgrad_3x3(int(sys.argv[2]) if len(sys.argv) > 2 else 1024)
    elif len(sys.argv) > 1 and sys.argv[1] == "--wgrad-s2d":
        wgrad_s2d(int(sys.argv[2]) if len(sys.argv) > 2 else 1024)
    else:
        run("stem7x7", 224, 8, 7, 2, 3)
        run("stem_s2d", 115, 16, 4, 1, 0)
