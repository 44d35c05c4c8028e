"""bench.py's exact ResNet-50 setup (MirroredStrategy scope, unseeded init, data seed 1234), eager vs captured:
per-step losses of both (debugging aid for the hipGraph path)."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    from distributed_tensorflow_amd import parallel
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=25)
    ap.add_argument("--jit", type=int, default=1)
    a = ap.parse_args()
    args = argparse.Namespace(model="resnet50", batch=256, lr=0.1, bucket_mb=None)
    strategy = parallel.MirroredStrategy()
    model, data, _, _ = bench.build(args, strategy, strategy.device, 0)
    model._jit = bool(a.jit)
    fn = model.make_train_function(force=True)
    out = []
    for _ in range(a.steps):
        out.append(float(fn(next(data))["loss"]))
    print("jit" if a.jit else "eager", " ".join(f"{v:.4f}" for v in out))


if __name__ == "__main__":
    main()
