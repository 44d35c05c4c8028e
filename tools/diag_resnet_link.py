"""Input-gradient error of the two-block ResNet test (tests/test_resnet_gpu.py::test_residual_grad_link_matches_reference)
against its bf16-storage CPU reference, per gradient, under the current environment (run it under different
DTF_* knobs to find which path moves the input gradient)."""
import sys

import torch

sys.path.insert(0, ".")
from tests import test_resnet_gpu as T  # noqa: E402
from distributed_tensorflow_amd import context, ops  # noqa: E402


def main():
    cuda = torch.device("cuda:0")
    g = torch.Generator().manual_seed(5)
    x = torch.randn(8, 16, 16, 64, generator=g)
    gb = T._blocks()
    run = T._run(gb, x.to(cuda).to(torch.bfloat16))
    real = ops.conv_bn
    ops.conv_bn = T._emu_conv_bn
    with context.device("cpu"):
        cb = T._blocks()
        with torch.no_grad():
            cb[0](torch.zeros(1, 16, 16, 64), training=False)
            cb[1](torch.zeros(1, 8, 8, 64), training=False)
        for vc, vg in zip([w for b in cb for w in b.trainable_weights], [w for b in gb for w in b.trainable_weights]):
            vc.data.copy_(vg.data.cpu())
        ref = T._run(cb, x.to(torch.bfloat16).float())
    ops.conv_bn = real
    errs, l2 = [], []
    for r, a in zip(ref, run):
        errs.append((a - r).abs().max().item() / (r.abs().max().item() + 1e-6))
        l2.append((a - r).norm().item() / (r.norm().item() + 1e-6))
    r, a = ref[0], run[0]
    d = (a - r).abs()
    idx = torch.nonzero(d == d.max())[0].tolist()
    # where is the x-gradient error: even/odd pixels (the stride-2 projection reads the even ones)
    ev = d[:, ::2, ::2].max().item() / r.abs().max().item()
    od = d[:, 1::2, :].max().item() / r.abs().max().item()
    print(f"x {errs[0]:.4f} (worst at {idx}, even-even pixels {ev:.4f}, odd rows {od:.4f}) "
          f"weights max {max(errs[1:]):.4f}; relative L2: x {l2[0]:.4f} worst {max(l2):.4f}", flush=True)


if __name__ == "__main__":
    main()
