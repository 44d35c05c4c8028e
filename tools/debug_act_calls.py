"""Which layers launch the standalone activation kernel (dtf_act) in a BERT-base training step: prints each call's
element count and the Python call site (bench config, batch 8). Usage: python tools/debug_act_calls.py"""
import collections
import os
import sys
import traceback

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from distributed_tensorflow_amd.keras import losses, optimizers  # noqa: E402
from distributed_tensorflow_amd.models.transformer import BertModel  # noqa: E402
from distributed_tensorflow_amd.ops import _util, conv, fp8, linalg, nn  # noqa: E402

seen = collections.Counter()


def wrap(mod):
    orig = mod.call

    def call(name, *args):
        if name == "dtf_act":
            site = traceback.extract_stack(limit=4)[-2]
            seen[(args[3], f"{os.path.basename(site.filename)}:{site.lineno}")] += 1
        return orig(name, *args)
    mod.call = call


for m in (linalg, nn, fp8, conv, _util):
    wrap(m)
dev = torch.device("cuda", 0)
model = BertModel()
model.compile(optimizer=optimizers.AdamW(1e-4, weight_decay=0.01, epsilon=1e-6),
              loss=losses.SparseCategoricalCrossentropy(from_logits=True))
B, S, P = 8, 512, 76
ids = torch.randint(0, 30522, (B, S), device=dev)
mpos = torch.stack([torch.randperm(S, device=dev)[:P] for _ in range(B)])
x = {"input_ids": ids, "masked_positions": mpos, "token_type_ids": torch.zeros_like(ids),
     "attention_mask": torch.ones(B, S, device=dev)}
lab = torch.randint(0, 30522, (B, P), device=dev)
for _ in range(2):
    model.train_step((x, lab))
torch.cuda.synchronize()
for (n, site), c in sorted(seen.items()):
    print(f"dtf_act n={n} x{c} at {site}")
