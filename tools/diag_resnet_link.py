"""Per-gradient relative error of the two ResNet block GPU paths (residual link off / on) against the bf16-storage
CPU reference of tests/test_resnet_gpu.py (diagnostic for test_residual_grad_link_matches_reference)."""
import sys

import torch

sys.path.insert(0, ".")
from tests import test_resnet_gpu as T  # noqa: E402
from distributed_tensorflow_amd import context, ops  # noqa: E402
from distributed_tensorflow_amd.models import resnet as R  # noqa: E402


def main():
    cuda = torch.device("cuda:0")
    g = torch.Generator().manual_seed(5)
    x = torch.randn(8, 16, 16, 64, generator=g)
    runs = {}
    for link in (False, True, False):
        R.RES_LINK = link
        gb = T._blocks()
        runs.setdefault(link, []).append(T._run(gb, x.to(cuda).to(torch.bfloat16)))
    R.RES_LINK = True
    real = ops.conv_bn
    ops.conv_bn = T._emu_conv_bn
    with context.device("cpu"):
        cb = T._blocks()
        with torch.no_grad():
            cb[0](torch.zeros(1, 16, 16, 64), training=False)
            cb[1](torch.zeros(1, 8, 8, 64), training=False)
        for vc, vg in zip([w for b in cb for w in b.trainable_weights], [w for b in gb for w in b.trainable_weights]):
            vc.data.copy_(vg.data.cpu())
        names = ["x"] + [w.name if hasattr(w, "name") else str(i) for i, w in
                         enumerate(w for b in cb for w in b.trainable_weights)]
        ref = T._run(cb, x.to(torch.bfloat16).float())
    ops.conv_bn = real
    for i, r in enumerate(ref):
        s = r.abs().max().item() + 1e-6
        e0 = (runs[False][0][i] - r).abs().max().item() / s
        e0b = (runs[False][1][i] - r).abs().max().item() / s
        e1 = (runs[True][0][i] - r).abs().max().item() / s
        same = torch.equal(runs[False][0][i], runs[False][1][i])
        print(f"{i:2d} {str(names[i])[:40]:40s} {tuple(r.shape)} plain {e0:.4f} plain2 {e0b:.4f} link {e1:.4f} "
              f"repeat-identical {same}", flush=True)


if __name__ == "__main__":
    main()
