#!/usr/bin/env python
"""GPT-2-medium loss trajectory, bf16 vs fp8 (fp8 forward + backward projections), same init / data / dropout
masks: python tools/fp8_loss_curve.py [steps] [batch]. Prints both curves and their max relative gap."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_tensorflow_amd.data import synthetic_tokens  # noqa: E402
from distributed_tensorflow_amd.keras import losses, optimizers  # noqa: E402
from distributed_tensorflow_amd.models.transformer import gpt2_medium  # noqa: E402
from distributed_tensorflow_amd.ops import mha as _mha, nn as _nn  # noqa: E402


def run(fp8, steps, batch):
    torch.manual_seed(0)
    _nn._seed_counter[0], _mha._seed_counter[0] = 0x5EED, 0
    dev = torch.device("cuda")
    model = gpt2_medium(fp8=fp8)
    model.compile(optimizer=optimizers.AdamW(3e-4, weight_decay=0.1),
                  loss=losses.SparseCategoricalCrossentropy(from_logits=True))
    data = iter(synthetic_tokens(batch, 1024, 50257, dev, seed=0))
    out = []
    for _ in range(steps):
        logs = model.train_step(next(data))
        out.append(float(logs["loss"]))
    return out


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    batch = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    a = run(False, steps, batch)
    b = run(True, steps, batch)
    gap = max(abs(x - y) / abs(x) for x, y in zip(a, b))
    print("step  bf16      fp8")
    for i, (x, y) in enumerate(zip(a, b)):
        print(f"{i:4d}  {x:.4f}  {y:.4f}")
    print(f"max relative gap {gap:.4f}; final bf16 {a[-1]:.4f} fp8 {b[-1]:.4f}")


if __name__ == "__main__":
    main()
