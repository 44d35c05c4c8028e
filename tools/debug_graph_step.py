"""Eager vs hipGraph-captured ResNet train steps at bench shape: per-step loss of both, first step where they
diverge, and which weights went non-finite.

    python tools/debug_graph_step.py [--batch 256] [--steps 8] [--opt sgd]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(jit, args):
    import torch
    from distributed_tensorflow_amd.data import synthetic_imagenet
    from distributed_tensorflow_amd.keras import initializers, losses, optimizers
    from distributed_tensorflow_amd.models import ResNet
    if not args.noseed:
        initializers.set_seed(3)
    dev = torch.device("cuda:0")
    model = ResNet(args.depth, num_classes=1000)
    opt = optimizers.SGD(args.lr, momentum=0.9) if args.opt == "sgd" else optimizers.Adam(1e-3)
    model.compile(optimizer=opt, loss=losses.SparseCategoricalCrossentropy(from_logits=True), jit_compile=jit)
    data = iter(synthetic_imagenet(args.batch, dev, seed=11))
    fn = model.make_train_function(force=True)
    out = []
    logs = None
    for _ in range(args.steps):
        logs = fn(next(data))
        if not args.nosync:
            out.append(float(logs["loss"]))
    torch.cuda.synchronize()
    if args.nosync:
        out.append(float(logs["loss"]))
    bad = [v.name for v in model.weights if not torch.isfinite(v.detach().float()).all()]
    return out, bad


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--depth", type=int, default=50)
    ap.add_argument("--lr", type=float, default=0.1)
    ap.add_argument("--opt", default="sgd")
    ap.add_argument("--nosync", action="store_true", help="read the loss only after the last step (bench.py)")
    ap.add_argument("--noseed", action="store_true")
    args = ap.parse_args()
    e, be = run(False, args)
    g, bg = run(True, args)
    print("eager:", " ".join(f"{v:.4f}" for v in e))
    print("graph:", " ".join(f"{v:.4f}" for v in g))
    print("non-finite eager:", be[:8], "graph:", bg[:8], len(bg))


if __name__ == "__main__":
    main()
