"""Stem kernel vs the implicit-GEMM conv on the bench shape (persistent blocks: several units per block) — output,
BN finalize outputs and running stats. python tools/debug_stem.py [N]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_tensorflow_amd.ops import conv as OC  # noqa: E402
from distributed_tensorflow_amd.ops._util import K, ptr, stream  # noqa: E402

BF = torch.bfloat16
dev = torch.device("cuda")
N = int(sys.argv[1]) if len(sys.argv) > 1 else 64
g = torch.Generator().manual_seed(5)
img = torch.randn(N, 3, 224, 224, generator=g).to(dev)
w7 = (torch.randn(64, 7, 7, 4, generator=g) * 0.05).to(dev)
x = OC.image_to_s2d_bf16(img)
w16 = OC.stem_s2d_filter(w7.to(BF))
res = []
for tile in (-1, 2):
    y = torch.empty(N, 112, 112, 64, dtype=BF, device=dev)
    part = torch.empty(((N * 112 * 112 + 63) // 64) * 128, device=dev)
    gamma = torch.ones(64, device=dev)
    beta = torch.zeros(64, device=dev)
    rm, rv = torch.zeros(64, device=dev), torch.ones(64, device=dev)
    outs = [torch.empty(64, device=dev) for _ in range(4)]
    rc = K().dtf_conv_fwd_bn(ptr(x), ptr(w16), ptr(y), ptr(part), N, 115, 115, 16, 64, 4, 4, 112, 112, 1, 1, 0, 0, 1,
                             1, tile, ptr(gamma), ptr(beta), ptr(rm), ptr(rv), 0.9, 1e-3, *[ptr(o) for o in outs], None,
                             None, None, stream())
    torch.cuda.synchronize()
    print("tile", tile, "rc", rc, flush=True)
    res.append((y.float(), [o.clone() for o in outs], rm.clone(), rv.clone()))
(y0, o0, m0, v0), (y1, o1, m1, v1) = res
print("y max diff", (y0 - y1).abs().max().item(), "max", y1.abs().max().item())
for name, a, b in zip(("scale", "shift", "mean", "invstd"), o0, o1):
    print(name, (a - b).abs().max().item(), b.abs().max().item())
print("rm", (m0 - m1).abs().max().item(), "rv", (v0 - v1).abs().max().item())
yf = y1.reshape(-1, 64)
print("true mean", (yf.mean(0) - o1[2]).abs().max().item(), (yf.mean(0) - o0[2]).abs().max().item())
