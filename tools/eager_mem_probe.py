"""Eager (uncaptured) ResNet-50 train steps at a given batch: host time per step and the caching allocator's
behaviour (cudaMalloc retries = the allocator freeing its cache to satisfy a request, peak reserved / allocated).

    python tools/eager_mem_probe.py [batch] [steps]
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_tensorflow_amd import parallel  # noqa: E402
from distributed_tensorflow_amd.keras import losses, optimizers  # noqa: E402
from distributed_tensorflow_amd.models import ResNet  # noqa: E402


def main():
    batch = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 6
    own_stream = len(sys.argv) > 3 and sys.argv[3] == "stream"
    dev = torch.device("cuda:0")
    if own_stream:  # issue on a created stream (as bench.py does) instead of the legacy default stream
        s = torch.cuda.Stream(device=dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        torch.cuda.set_stream(s)
    strategy = parallel.MirroredStrategy()
    with strategy.scope():
        model = ResNet(50, num_classes=1000)
        model.compile(optimizer=optimizers.SGD(0.1, momentum=0.9),
                      loss=losses.SparseCategoricalCrossentropy(from_logits=True))
    x = torch.randn(batch, 3, 224, 224, device=dev)
    y = torch.randint(0, 1000, (batch,), device=dev)
    fn = model.make_train_function(force=True)
    for i in range(steps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn((x, y))
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        st = torch.cuda.memory_stats(dev)
        print(f"step {i}: issue {1e3 * (t1 - t0):8.1f} ms  total {1e3 * (t2 - t0):8.1f} ms  "
              f"retries {st.get('num_alloc_retries', 0)}  hipMalloc {st.get('num_device_alloc', 0)}  "
              f"peak alloc {st['allocated_bytes.all.peak'] / 2**30:6.1f} GiB  reserved {st['reserved_bytes.all.current'] / 2**30:6.1f} GiB",
              flush=True)


if __name__ == "__main__":
    main()
