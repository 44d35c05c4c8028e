"""One SGD(lr=1) step of a reduced ResNet on the GPU path vs the bf16-emulating CPU reference: the per-parameter
relative difference of the update (= -gradient), worst first (debugging aid for tests/test_model_training_gpu.py)."""
import sys
sys.path.insert(0, "/root/repo")
sys.path.insert(0, "/root/repo/tests")
import numpy as np  # noqa: E402
import torch  # noqa: E402
from distributed_tensorflow_amd import context, ops  # noqa: E402
from distributed_tensorflow_amd.keras import initializers, losses, optimizers  # noqa: E402
from distributed_tensorflow_amd.models import ResNet  # noqa: E402
import distributed_tensorflow_amd.ops.conv as OC  # noqa: E402


def grads(dev, x, y):
    with context.device(dev):
        initializers.set_seed(11)
        m = ResNet(26, num_classes=10, width=16)
        m.compile(optimizer=optimizers.SGD(1.0), loss=losses.SparseCategoricalCrossentropy(from_logits=True))
        with torch.no_grad():
            m(x.to(dev)[:1], training=False)
        before = [w.detach().float().cpu().clone() for w in m.weights]
        loss = float(m.train_step((x.to(dev), y.to(dev)))["loss"])
        after = [w.detach().float().cpu().clone() for w in m.weights]
    return loss, [(b - a) for a, b in zip(after, before)], [w.name for w in m.weights]


def compare(a_list, b_list, names, top=8, label=""):
    rows = []
    for n, a, b in zip(names, a_list, b_list):
        if b.numel() < 2:
            continue
        rows.append((float((a - b).norm() / (b.norm() + 1e-12)), n))
    rows.sort(reverse=True)
    print(label, "median rel", round(float(np.median([r[0] for r in rows])), 4), "worst", rows[:3])


for batch, hw in ((8, 64), (32, 96)):
    g = torch.Generator().manual_seed(0)
    x, y = torch.randn(batch, 3, hw, hw, generator=g), torch.randint(0, 10, (batch,), generator=g)
    lg, dg, names = grads(torch.device("cuda:0"), x, y)
    lp, dp, _ = grads(torch.device("cuda:0"), x + 1e-3 * torch.randn(x.shape, generator=g), y)
    import test_resnet_gpu as emu  # noqa: E402
    c0, c1 = ops.conv_bn, OC.conv_bn
    ops.conv_bn = emu._emu_conv_bn
    OC.conv_bn = emu._emu_conv_bn
    lc, dc, _ = grads(torch.device("cpu"), x, y)
    lc2, dc2, _ = grads(torch.device("cpu"), x + 1e-3 * torch.randn(x.shape, generator=g), y)
    ops.conv_bn, OC.conv_bn = c0, c1
    print(f"batch {batch} {hw}x{hw}: loss gpu {lg:.5f} cpu {lc:.5f}")
    compare(dg, dc, names, label="  gpu vs cpu-emu        ")
    compare(dg, dp, names, label="  gpu vs gpu(x+1e-3 nz) ")
    compare(dc, dc2, names, label="  cpu vs cpu(x+1e-3 nz) ")
