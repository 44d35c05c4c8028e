import sys, torch
sys.path.insert(0, ".")
from tests.test_resnet_gpu import _grads, _model
from distributed_tensorflow_amd.models import resnet as R
from distributed_tensorflow_amd import context
cuda = torch.device("cuda")
g = torch.Generator().manual_seed(5)
x = torch.randn(4, 3, 64, 64, generator=g)
y = torch.randint(0, 10, (4,), generator=g)
gm = _model()
a = _grads(gm, x.to(cuda), y.to(cuda))
names = [v.name for v in gm.trainable_weights]
with context.device("cpu"):
    cm = _model()
    with torch.no_grad():
        cm(x, training=False)
    for vc, vg in zip(cm.trainable_weights, gm.trainable_weights):
        vc.data.copy_(vg.data.cpu())
    ref = _grads(cm, x, y)
for i, (r, b, n) in enumerate(zip(ref, a, names)):
    s = r.abs().max().item() + 1e-6
    print(i, n, tuple(r.shape), f"|ref| {s:.3e} |gpu| {b.abs().max().item():.3e} err {(b - r).abs().max().item() / s:.2e}")
