"""Calibration for tests/test_model_training_gpu.py: one SGD(lr=1) step of a reduced ResNet on the
GPU path vs the bf16-emulating CPU reference, per-parameter relative difference of the update (= -gradient), for
several batch / image sizes and label kinds (random vs a fixed learnable teacher), next to the CPU reference's own
sensitivity to a 1e-3 input perturbation."""
import sys
sys.path.insert(0, "/root/repo")
sys.path.insert(0, "/root/repo/tests")
import numpy as np  # noqa: E402
import torch  # noqa: E402
from distributed_tensorflow_amd import context, ops  # noqa: E402
from distributed_tensorflow_amd.keras import initializers, losses, optimizers  # noqa: E402
from distributed_tensorflow_amd.models import ResNet  # noqa: E402
import distributed_tensorflow_amd.ops.conv as OC  # noqa: E402


def grads(dev, x, y, depth, width):
    with context.device(dev):
        initializers.set_seed(11)
        m = ResNet(depth, num_classes=10, width=width)
        m.compile(optimizer=optimizers.SGD(1.0), loss=losses.SparseCategoricalCrossentropy(from_logits=True))
        with torch.no_grad():
            m(x.to(dev)[:1], training=False)
        before = [w.detach().float().cpu().clone() for w in m.weights]
        loss = float(m.train_step((x.to(dev), y.to(dev)))["loss"])
        after = [w.detach().float().cpu().clone() for w in m.weights]
    return loss, [(b - a) for a, b in zip(after, before)]


def med(a_list, b_list):
    r = [float((a - b).norm() / (b.norm() + 1e-12)) for a, b in zip(a_list, b_list) if b.numel() > 1]
    return float(np.median(r)), float(np.percentile(r, 90))


import test_resnet_gpu as emu  # noqa: E402
for depth, width, batch, hw, lab in ((26, 16, 8, 64, "rand"), (26, 16, 8, 64, "teacher"), (26, 16, 32, 64, "teacher"),
                                     (26, 32, 32, 64, "teacher"), (26, 16, 32, 96, "teacher")):
    g = torch.Generator().manual_seed(0)
    x = torch.randn(batch, 3, hw, hw, generator=g)
    if lab == "rand":
        y = torch.randint(0, 10, (batch,), generator=g)
    else:  # a fixed linear teacher on the 4x4-pooled image: learnable labels
        t = torch.randn(3 * 16, 10, generator=torch.Generator().manual_seed(99))
        y = (torch.nn.functional.adaptive_avg_pool2d(x, 4).flatten(1) @ t).argmax(1)
    noise = 1e-3 * torch.randn(x.shape, generator=g)
    lg, dg = grads(torch.device("cuda:0"), x, y, depth, width)
    orig = (ops.conv_bn, OC.conv_bn)
    ops.conv_bn, OC.conv_bn = emu._emu_conv_bn, emu._emu_conv_bn
    lc, dc = grads(torch.device("cpu"), x, y, depth, width)
    _, dc2 = grads(torch.device("cpu"), x + noise, y, depth, width)
    ops.conv_bn, OC.conv_bn = orig
    e, s = med(dg, dc), med(dc2, dc)
    print(f"resnet{depth} w{width} b{batch} {hw}px {lab:7s}: loss gpu {lg:.5f} cpu {lc:.5f} | gpu-vs-cpu median "
          f"{e[0]:.4f} p90 {e[1]:.4f} | cpu sensitivity median {s[0]:.4f} p90 {s[1]:.4f}", flush=True)

# frozen (inference-mode) BatchNorm: the well-conditioned comparison of tests/test_model_training_gpu.py
import test_model_training_gpu as tm  # noqa: E402
g = torch.Generator().manual_seed(0)
x = torch.randn(8, 3, 64, 64, generator=g)
t = torch.randn(3 * 16, 10, generator=torch.Generator().manual_seed(99))
y = (torch.nn.functional.adaptive_avg_pool2d(x, 4).flatten(1) @ t).argmax(1)
orig = (ops.conv_bn, OC.conv_bn)
ops.conv_bn, OC.conv_bn = emu._emu_conv_bn, emu._emu_conv_bn
lc, gc, wc = tm._frozen_bn_grads(torch.device("cpu"), x, y)
_, gc2, _ = tm._frozen_bn_grads(torch.device("cpu"), x + 1e-3 * torch.randn(x.shape, generator=g), y)
ops.conv_bn, OC.conv_bn = orig
lg, gg, _ = tm._frozen_bn_grads(torch.device("cuda:0"), x, y, ref_weights=wc)
e, s = med(gg, gc), med(gc2, gc)
print(f"frozen-BN resnet26 w16 b8 64px teacher: loss gpu {lg:.5f} cpu {lc:.5f} | gpu-vs-cpu median {e[0]:.4f} p90 "
      f"{e[1]:.4f} | cpu sensitivity (1e-3) median {s[0]:.4f} p90 {s[1]:.4f}", flush=True)
