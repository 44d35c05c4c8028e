import sys, torch
sys.path.insert(0, ".")
import tests.test_resnet_gpu as T
from distributed_tensorflow_amd import context
cuda = torch.device("cuda")
g = torch.Generator().manual_seed(5)
x = torch.randn(8, 16, 16, 64, generator=g)
gb = T._blocks()
a = T._run(gb, x.to(cuda).to(torch.bfloat16))
names = ["x"] + [w.name for b in gb for w in b.trainable_weights]
with context.device("cpu"):
    cb = T._blocks()
    with torch.no_grad():
        cb[0](torch.zeros(1, 16, 16, 64), training=False)
        cb[1](torch.zeros(1, 8, 8, 64), training=False)
    for vc, vg in zip([w for b in cb for w in b.trainable_weights], [w for b in gb for w in b.trainable_weights]):
        vc.data.copy_(vg.data.cpu())
    ref = T._run(cb, x.to(torch.bfloat16).float())
for n, r, b in zip(names, ref, a):
    s = r.abs().max().item() + 1e-6
    print(n, tuple(r.shape), f"|ref| {s:.3e} err {(b - r).abs().max().item() / s:.2e} mean-rel {((b-r).abs().mean() / r.abs().mean()).item():.2e}")
