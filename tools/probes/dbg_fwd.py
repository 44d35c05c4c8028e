import sys, torch
sys.path.insert(0, ".")
from tests.test_resnet_gpu import _model
from distributed_tensorflow_amd import context, ops
cuda = torch.device("cuda")
g = torch.Generator().manual_seed(5)
x = torch.randn(4, 3, 64, 64, generator=g)
gm = _model()
with torch.no_grad():
    gm(x.to(cuda), training=False)
with context.device("cpu"):
    cm = _model()
    with torch.no_grad():
        cm(x, training=False)
    for vc, vg in zip(cm.weights, gm.weights):
        vc.data.copy_(vg.data.cpu())

def trace(m, xin):
    out = []
    h = ops.image_to_nhwc_bf16(xin, m.in_pad)
    out.append(("in", h))
    h = m.stem(h, training=True); out.append(("stem", h))
    h = m.pool(h); out.append(("pool", h))
    for i, b in enumerate(m.blocks):
        y1 = b.c1(h, training=True); out.append((f"b{i}.c1", y1))
        y2 = b.c2(y1, training=True); out.append((f"b{i}.c2", y2))
        sc = b.proj(h, training=True) if b.proj is not None else h
        if b.proj is not None: out.append((f"b{i}.proj", sc))
        h = b.c3(y2, residual=sc, training=True); out.append((f"b{i}.out", h))
    return out

with torch.no_grad():
    tg = trace(gm, x.to(cuda))
    with context.device("cpu"):
        tc = trace(cm, x)
for (n, a), (_, b) in zip(tg, tc):
    a = a.float().cpu(); b = b.float()
    s = b.abs().max().item() + 1e-6
    print(n, tuple(a.shape), tuple(b.shape), f"rel err {(a - b).abs().max().item() / s:.3e}  mean abs err {(a-b).abs().mean().item():.3e}")
