"""Per-layer roofline of ResNet-50's convolutions (batch 256, bf16 NHWC) through our implicit-GEMM kernels.

For every distinct conv of ResNet-50 v1.5 (with its multiplicity in the network) times forward (with the BN
statistics epilogue, as the model runs it), data gradient and weight gradient (accumulating into an f32
arena view) for the default tile choice and each forced tile, and prints achieved TFLOP/s next to the two
floors: HBM bytes at 5 TB/s and FLOPs at 1.3 PFLOP/s (a practical MFMA rate). Totals are weighted by
multiplicity, so the last lines say how much of the step the GEMM side could still give back.

  python tools/conv_roofline.py [--tiles] [--only fwd|dgrad|wgrad]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_tensorflow_amd.ops import conv as C  # noqa: E402
from distributed_tensorflow_amd.ops._util import IntOut, call, ptr, stream, workspace  # noqa: E402

BF = torch.bfloat16
NB = 256
TILES = None


def layers():
    """(name, H, Cin, K, R, stride, count): ResNet-50 v1.5 convs, input spatial H."""
    out = [("stem7x7", 224, 8, 64, 7, 2, 1)]
    H = 56
    cin = 64
    for si, (n, w) in enumerate(zip((3, 4, 6, 3), (64, 128, 256, 512))):
        s = 1 if si == 0 else 2
        Ho = H // s
        out.append((f"s{si + 1}b0.c1", H, cin, w, 1, 1, 1))
        out.append((f"s{si + 1}b0.c2", H, w, w, 3, s, 1))
        out.append((f"s{si + 1}b0.c3", Ho, w, 4 * w, 1, 1, 1))
        out.append((f"s{si + 1}b0.proj", H, cin, 4 * w, 1, s, 1))
        out.append((f"s{si + 1}bX.c1", Ho, 4 * w, w, 1, 1, n - 1))
        out.append((f"s{si + 1}bX.c2", Ho, w, w, 3, 1, n - 1))
        out.append((f"s{si + 1}bX.c3", Ho, w, 4 * w, 1, 1, n - 1))
        H, cin = Ho, 4 * w
    return out


def timeit(fn, iters=10, warm=2):
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
    ap = argparse.ArgumentParser()
    ap.add_argument("--tiles", action="store_true", help="also time every forced tile shape")
    ap.add_argument("--only", default=None)
    ap.add_argument("--tile-list", default=None, help="comma-separated tiles for --tiles")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--match", default=None, help="only layers whose name contains this")
    args = ap.parse_args()
    global TILES, NB
    NB = args.batch
    TILES = [int(t) for t in args.tile_list.split(",")] if args.tile_list else None
    dev = torch.device("cuda")
    torch.manual_seed(0)
    tot = {"fwd": [0.0, 0.0, 0.0], "dgrad": [0.0, 0.0, 0.0], "wgrad": [0.0, 0.0, 0.0]}
    for name, H, Cin, K, R, s, cnt in layers():
        if args.match and args.match not in name:
            continue
        p = R // 2
        x = torch.randn(NB, H, H, Cin, device=dev).to(BF)
        w = torch.randn(K, R, R, Cin, device=dev) * 0.05
        w16 = w.to(BF)
        g = C._geom(x, w, (s, s), (p, p), (1, 1))
        N_, H_, W_, C_, K_, R_, S_, P, Q, *_ = g
        dy = torch.randn(NB, P, Q, K, device=dev).to(BF)
        M = NB * P * Q
        fl = 2.0 * M * K * R * R * Cin
        xb, yb = x.numel() * 2, dy.numel() * 2
        ws = workspace(dev)
        dwacc = torch.zeros(K, R, R, Cin, device=dev)
        part = torch.empty(((M + 63) // 64) * 2 * K, dtype=torch.float32, device=dev)
        rows = IntOut()
        y = torch.empty(NB, P, Q, K, device=dev, dtype=BF)
        dx = torch.empty_like(x)
        wc = C.crsk_shadow(w, K, R * R, Cin)

        def fwd(tile):
            return lambda: call("dtf_conv_fwd", ptr(x), ptr(w16), ptr(y), None, ptr(part), rows.addr, NB, H, H, Cin,
                                K, R, R, P, Q, s, s, p, p, 1, 1, 0, 0, tile, stream())

        def dgrad(tile):
            return lambda: call("dtf_conv_dgrad", ptr(dy), ptr(wc), ptr(dx), NB, H, H, Cin, K, R, R, P, Q, s, s, p, p,
                                1, 1, 0, 0.0, tile, ptr(ws), 2 * ws.numel(), None, None, None, None, None, None,
                                stream())

        def wgrad(tile):
            return lambda: call("dtf_conv_wgrad", ptr(x), ptr(dy), ptr(dwacc), NB, H, H, Cin, K, R, R, P, Q, s, s, p,
                                p, 1, 1, 1, 0, tile, ptr(ws), ws.numel(), stream())

        for kind, mk, byts in (("fwd", fwd, xb + yb), ("dgrad", dgrad, xb + yb), ("wgrad", wgrad, xb + yb)):
            if args.only and kind != args.only:
                continue
            t = timeit(mk(-1))
            floor = max(byts / 5e12, fl / 1.3e15)
            line = (f"{name:12s} x{cnt} {kind:5s} M={M:7d} N={K if kind != 'dgrad' else Cin:5d} "
                    f"{t * 1e6:7.1f}us {fl / t / 1e12:6.0f}TF {byts / t / 1e12:5.2f}TB/s floor={floor * 1e6:6.1f}us "
                    f"({'mem' if byts / 5e12 > fl / 1.3e15 else 'mfma'}) x{t / floor:4.1f}")
            best = t
            if args.tiles:
                for tile in (TILES or range(0, 11)):
                    try:
                        tt = timeit(mk(tile))
                    except Exception:  # noqa: BLE001 - tile not instantiated for this mode
                        continue
                    best = min(best, tt)
                    line += f" t{tile}:{tt * 1e6:.0f}"
            print(line, flush=True)
            tot[kind][0] += cnt * t
            tot[kind][1] += cnt * best
            tot[kind][2] += cnt * floor
    allt = [0.0, 0.0, 0.0]
    for kind, (t, b, f) in tot.items():
        print(f"TOTAL {kind:5s}: {t * 1e3:6.2f} ms (best tile {b * 1e3:6.2f} ms, floor {f * 1e3:6.2f} ms)")
        for i, v in enumerate((t, b, f)):
            allt[i] += v
    print(f"TOTAL all  : {allt[0] * 1e3:6.2f} ms (best tile {allt[1] * 1e3:6.2f} ms, floor {allt[2] * 1e3:6.2f} ms)")


if __name__ == "__main__":
    main()
