"""Per-step training loss of a bench model (same build as bench.py): python tools/debug_loss_steps.py [model] [steps]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("GPU_MAX_HW_QUEUES", "8")
import bench  # noqa: E402
import torch  # noqa: E402
from distributed_tensorflow_amd import parallel  # noqa: E402

m = sys.argv[1] if len(sys.argv) > 1 else "resnet50"
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 8
args = argparse.Namespace(model=m, batch=bench.DEFAULT_BATCH[m], lr=0.1)
strategy = parallel.MirroredStrategy()
model, data, _, _ = bench.build(args, strategy, strategy.device, 0)
fn = model.make_train_function(force=True)
for i in range(steps):
    logs = fn(next(data))
    print(i, round(float(logs["loss"]), 5), flush=True)
