"""ResNet-50 1x1 convolutions (batch 256) as plain GEMMs: our implicit-GEMM conv kernels (with the BN-statistics
epilogue the model uses in the forward) vs hipBLASLt (torch.mm) on the same shapes — how far the MFMA kernels
are from the library GEMM on each layer.

  python tools/bench_blas_conv1x1.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_tensorflow_amd.ops import conv as C  # noqa: E402
from distributed_tensorflow_amd.ops._util import IntOut, call, ptr, stream, workspace  # noqa: E402
from tools.conv_roofline import timeit  # noqa: E402

BF = torch.bfloat16
dev = torch.device("cuda")
for (H, Cin, K) in [(56, 64, 256), (56, 256, 64), (28, 128, 512), (28, 512, 128), (14, 256, 1024), (14, 1024, 256),
                    (7, 512, 2048), (7, 2048, 512)]:
    N = 256
    M = N * H * H
    x = torch.randn(N, H, H, Cin, device=dev).to(BF)
    w = torch.randn(K, 1, 1, Cin, device=dev) * 0.05
    w16 = w.to(BF)
    g = C._geom(x, w, (1, 1), (0, 0), (1, 1))
    y = torch.empty(N, H, H, K, device=dev, dtype=BF)
    part = torch.empty(((M + 63) // 64) * 2 * K, dtype=torch.float32, device=dev)
    rows = IntOut()
    dy = torch.randn(N, H, H, K, device=dev).to(BF)
    dx = torch.empty_like(x)
    ws = workspace(dev)
    wc = C.crsk_shadow(w, K, 1, Cin)
    dwacc = torch.zeros(K, 1, 1, Cin, device=dev)
    fl = 2.0 * M * K * Cin
    t_f = timeit(lambda: call("dtf_conv_fwd", ptr(x), ptr(w16), ptr(y), None, ptr(part), rows.addr, N, H, H, Cin, K,
                              1, 1, H, H, 1, 1, 0, 0, 1, 1, 0, 0, -1, stream()))
    t_fb = timeit(lambda: torch.mm(x.view(M, Cin), w16.view(K, Cin).t()))
    t_d = timeit(lambda: call("dtf_conv_dgrad", ptr(dy), ptr(wc), ptr(dx), N, H, H, Cin, K, 1, 1, H, H, 1, 1, 0, 0, 1,
                              1, 0, 0.0, -1, ptr(ws), 2 * ws.numel(), None, None, None, None, None, None, stream()))
    t_db = timeit(lambda: torch.mm(dy.view(M, K), w16.view(K, Cin)))
    t_w = timeit(lambda: call("dtf_conv_wgrad", ptr(x), ptr(dy), ptr(dwacc), N, H, H, Cin, K, 1, 1, H, H, 1, 1, 0, 0,
                              1, 1, 1, 0, -1, ptr(ws), ws.numel(), stream()))
    t_wb = timeit(lambda: torch.mm(dy.view(M, K).t(), x.view(M, Cin), out_dtype=torch.float32))
    print(f"H={H:3d} C={Cin:5d} K={K:5d}  fwd+stats ours {t_f * 1e6:6.1f}us blas {t_fb * 1e6:6.1f}us | dgrad ours "
          f"{t_d * 1e6:6.1f}us blas {t_db * 1e6:6.1f}us | wgrad ours {t_w * 1e6:6.1f}us blas(f32) {t_wb * 1e6:6.1f}us",
          flush=True)
