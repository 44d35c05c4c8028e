#!/usr/bin/env python
"""Host-side cost of one ResNet-50 b256 training step: the CPU time to ISSUE a step (train_fn returns without any
device sync) vs the device time per step, and the top Python hotspots of the issue path (cProfile). When the issue
time approaches the device time the GPU starves wherever the host has extra work (step start, loss -> backward).

    python tools/cpu_issue_time.py [--steps 10] [--profile]
"""
import argparse
import cProfile
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("GPU_MAX_HW_QUEUES", "8")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--profile", action="store_true")
    args = ap.parse_args()
    import torch
    import bench
    from distributed_tensorflow_amd import parallel
    strategy = parallel.MirroredStrategy()
    ns = argparse.Namespace(model="resnet50", batch=256, lr=0.1, graph=0)
    model, data, unit, cfg = bench.build(ns, strategy, strategy.device, 0)
    fn = model.make_train_function(force=True)
    for _ in range(5):
        x, y = next(data)
        fn((x, y))
    torch.cuda.synchronize()
    issue = []
    t0 = time.perf_counter()
    pr = cProfile.Profile() if args.profile else None
    for _ in range(args.steps):
        x, y = next(data)
        a = time.perf_counter()
        if pr:
            pr.enable()
        fn((x, y))
        if pr:
            pr.disable()
        issue.append(time.perf_counter() - a)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / args.steps
    print(f"issue per step: mean {1e3 * sum(issue) / len(issue):.2f} ms (min {1e3 * min(issue):.2f}, max "
          f"{1e3 * max(issue):.2f}); wall per step {1e3 * wall:.2f} ms", flush=True)
    if pr:
        st = pstats.Stats(pr)
        st.sort_stats("tottime").print_stats(25)


if __name__ == "__main__":
    main()
