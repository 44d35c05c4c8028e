"""Attribute the non-framework device work of one training step (runtime copies, fills, at::native kernels)
to the Python call sites that issue it: torch.profiler over one warm step, grouped by op name and the
innermost framework stack frame.

    python tools/attribute_step_ops.py [--model resnet50] [--batch 256] [--graph 0]
"""
import argparse
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--batch", type=int, default=256)
    args = ap.parse_args()
    import torch
    from torch.profiler import ProfilerActivity, profile

    from distributed_tensorflow_amd.data import synthetic_imagenet
    from distributed_tensorflow_amd.keras import losses, optimizers
    from distributed_tensorflow_amd.models import ResNet

    dev = torch.device("cuda:0")
    model = ResNet(int(args.model[6:]), num_classes=1000)
    model.compile(optimizer=optimizers.SGD(0.1, momentum=0.9),
                  loss=losses.SparseCategoricalCrossentropy(from_logits=True))
    data = iter(synthetic_imagenet(args.batch, dev, seed=1))
    fn = model.make_train_function(force=True)
    for _ in range(3):
        fn(next(data))
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
        fn(next(data))
        torch.cuda.synchronize()
    interesting = ("aten::copy_", "aten::to", "aten::_to_copy", "aten::fill_", "aten::zero_", "aten::cat",
                   "aten::add_", "aten::add", "aten::index_select", "aten::scatter", "aten::gather", "aten::mean",
                   "aten::sum", "aten::clone", "aten::contiguous", "aten::mul", "aten::div", "aten::item",
                   "aten::_local_scalar_dense", "aten::zeros", "aten::ones", "aten::full", "aten::lt", "aten::eq")
    by_site = collections.Counter()
    for ev in prof.events():
        if ev.name not in interesting:
            continue
        frames = [f for f in (ev.stack or []) if "distributed_tensorflow_amd" in f or "tools/" in f]
        site = frames[0] if frames else "<no framework frame>"
        by_site[(ev.name, site)] += 1
    print("== aten ops by innermost framework frame (count per step) ==")
    for (name, site), n in sorted(by_site.items(), key=lambda kv: -kv[1]):
        print(f"{n:5d}  {name:28s} {site}")
    print("== device kernels (count, total us) ==")
    kern = collections.defaultdict(lambda: [0, 0.0])
    for ev in prof.events():
        if ev.device_type == torch.autograd.DeviceType.CUDA:
            k = kern[ev.name[:110]]
            k[0] += 1
            k[1] += ev.device_time_total if hasattr(ev, "device_time_total") else ev.cuda_time_total
    for name, (n, us) in sorted(kern.items(), key=lambda kv: -kv[1][1])[:60]:
        print(f"{n:5d} {us:10.1f}  {name}")


if __name__ == "__main__":
    main()
