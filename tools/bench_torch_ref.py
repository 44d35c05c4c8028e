"""Vendor-library comparison point: the same ResNet-50 v1.5 training step written in plain
PyTorch (channels_last, bf16 autocast; MIOpen convs, hipBLASLt FC, PyTorch BN/SGD) on the same GPU.

  python tools/bench_torch_ref.py --batch 256 --steps 10 --warmup 3
"""
import argparse
import json
import time

import torch
import torch.nn as nn


class Bottleneck(nn.Module):
    def __init__(self, cin, w, stride, project):
        super().__init__()
        self.c1 = nn.Conv2d(cin, w, 1, bias=False)
        self.b1 = nn.BatchNorm2d(w)
        self.c2 = nn.Conv2d(w, w, 3, stride, 1, bias=False)
        self.b2 = nn.BatchNorm2d(w)
        self.c3 = nn.Conv2d(w, 4 * w, 1, bias=False)
        self.b3 = nn.BatchNorm2d(4 * w)
        self.proj = nn.Sequential(nn.Conv2d(cin, 4 * w, 1, stride, bias=False), nn.BatchNorm2d(4 * w)) \
            if project else None

    def forward(self, x):
        sc = self.proj(x) if self.proj is not None else x
        y = torch.relu(self.b1(self.c1(x)))
        y = torch.relu(self.b2(self.c2(y)))
        return torch.relu(self.b3(self.c3(y)) + sc)


class ResNet50(nn.Module):
    def __init__(self):
        super().__init__()
        self.stem = nn.Sequential(nn.Conv2d(3, 64, 7, 2, 3, bias=False), nn.BatchNorm2d(64), nn.ReLU(),
                                  nn.MaxPool2d(3, 2, 1))
        blocks, cin = [], 64
        for si, n in enumerate((3, 4, 6, 3)):
            w = 64 * 2 ** si
            for bi in range(n):
                blocks.append(Bottleneck(cin, w, 2 if (bi == 0 and si > 0) else 1, bi == 0))
                cin = 4 * w
        self.blocks = nn.Sequential(*blocks)
        self.fc = nn.Linear(2048, 1000)

    def forward(self, x):
        x = self.blocks(self.stem(x))
        return self.fc(torch.flatten(nn.functional.adaptive_avg_pool2d(x, 1), 1))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    a = ap.parse_args()
    torch.backends.cudnn.benchmark = True
    dev = torch.device("cuda")
    m = ResNet50().to(dev).to(memory_format=torch.channels_last)
    opt = torch.optim.SGD(m.parameters(), lr=0.1, momentum=0.9)
    x = torch.randn(a.batch, 3, 224, 224, device=dev).to(memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (a.batch,), device=dev)

    def step():
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = nn.functional.cross_entropy(m(x), y)
        opt.zero_grad(set_to_none=True)
        loss.backward()
        opt.step()
        return loss

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(a.steps):
        loss = step()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t
    print(json.dumps({"impl": "pytorch+MIOpen (channels_last, bf16 autocast)", "images_per_sec": a.batch * a.steps / dt,
                      "ms_per_step": dt / a.steps * 1e3, "loss": float(loss)}))


if __name__ == "__main__":
    main()
