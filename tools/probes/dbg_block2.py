import sys, torch
sys.path.insert(0, ".")
import tests.test_resnet_gpu as T
from distributed_tensorflow_amd import context, ops
from distributed_tensorflow_amd.ops import conv as OC
from distributed_tensorflow_amd.ops.norm import batch_norm_ref

class _Rnd(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x): return x.to(torch.bfloat16).float()
    @staticmethod
    def backward(ctx, g): return g.to(torch.bfloat16).float()
rnd = _Rnd.apply
def emu_conv_bn(x, w, gamma, beta, rmean, rvar, stride=(1, 1), pad=(0, 0), dil=(1, 1), relu=True, residual=None,
                momentum=0.9, eps=1e-5, training=True, link=None, role=None):
    y = rnd(OC._ref_conv(rnd(x), rnd(w), None, tuple(stride), tuple(pad), tuple(dil)))
    y = batch_norm_ref(y, gamma, beta, rmean, rvar, momentum, eps, training)
    if residual is not None:
        y = y + rnd(residual)
    if relu:
        y = torch.relu(y)
    return rnd(y)

cuda = torch.device("cuda")
g = torch.Generator().manual_seed(5)
x = torch.randn(8, 16, 16, 64, generator=g)
gb = T._blocks()
a = T._run(gb, x.to(cuda).to(torch.bfloat16))
names = ["x"] + [w.name for b in gb for w in b.trainable_weights]
res = {}
for emu in (False, True):
    if emu:
        ops.conv_bn = emu_conv_bn
    with context.device("cpu"):
        cb = T._blocks()
        with torch.no_grad():
            cb[0](torch.zeros(1, 16, 16, 64), training=False)
            cb[1](torch.zeros(1, 8, 8, 64), training=False)
        for vc, vg in zip([w for b in cb for w in b.trainable_weights], [w for b in gb for w in b.trainable_weights]):
            vc.data.copy_(vg.data.cpu())
        res[emu] = T._run(cb, x.to(torch.bfloat16).float())
for n, r, re, b in zip(names, res[False], res[True], a):
    s = r.abs().max().item() + 1e-6
    print(n, tuple(r.shape), f"gpu-vs-f32 {(b - r).abs().max().item() / s:.2e} gpu-vs-emu {(b - re).abs().max().item() / s:.2e} emu-vs-f32 {(re - r).abs().max().item() / s:.2e}")
