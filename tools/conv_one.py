"""Run ONE ResNet-50 conv (by layer name from conv_roofline.layers) fwd|dgrad|wgrad N times: a short target for
rocprofv3 --pmc passes.   python tools/conv_one.py s3bX.c2 fwd [iters] [tile]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import conv_roofline as R  # noqa: E402
from distributed_tensorflow_amd.ops import conv as C  # noqa: E402
from distributed_tensorflow_amd.ops._util import IntOut, call, ptr, stream, workspace  # noqa: E402

name, kind = sys.argv[1], sys.argv[2]
iters = int(sys.argv[3]) if len(sys.argv) > 3 else 20
tile = int(sys.argv[4]) if len(sys.argv) > 4 else -1
L = {l[0]: l for l in R.layers()}[name]
_, H, Cin, K, Rk, s, _ = L
p = Rk // 2
dev = torch.device("cuda")
NB = R.NB
x = torch.randn(NB, H, H, Cin, device=dev).to(torch.bfloat16)
w = torch.randn(K, Rk, Rk, Cin, device=dev) * 0.05
w16 = w.to(torch.bfloat16)
g = C._geom(x, w, (s, s), (p, p), (1, 1))
P, Q = g[7], g[8]
dy = torch.randn(NB, P, Q, K, device=dev).to(torch.bfloat16)
M = NB * P * Q
ws = workspace(dev)
dwacc = torch.zeros(K, Rk, Rk, Cin, device=dev)
part = torch.empty(((M + 63) // 64) * 2 * K, dtype=torch.float32, device=dev)
rows = IntOut()
y = torch.empty(NB, P, Q, K, device=dev, dtype=torch.bfloat16)
dx = torch.empty_like(x)
wc = C.crsk_shadow(w, K, Rk * Rk, Cin)
for _ in range(iters):
    if kind == "fwd":
        call("dtf_conv_fwd", ptr(x), ptr(w16), ptr(y), None, ptr(part), rows.addr, NB, H, H, Cin, K, Rk, Rk, P, Q, s, s,
             p, p, 1, 1, 0, 0, tile, stream())
    elif kind == "dgrad":
        call("dtf_conv_dgrad", ptr(dy), ptr(wc), ptr(dx), NB, H, H, Cin, K, Rk, Rk, P, Q, s, s, p, p, 1, 1, 0, 0.0, tile,
             ptr(ws), 2 * ws.numel(), None, None, None, None, None, None, stream())
    else:
        call("dtf_conv_wgrad", ptr(x), ptr(dy), ptr(dwacc), NB, H, H, Cin, K, Rk, Rk, P, Q, s, s, p, p, 1, 1, 1, 0, tile,
             ptr(ws), ws.numel(), stream())
torch.cuda.synchronize()
print("done", name, kind, M)
