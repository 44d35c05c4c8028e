"""One task of a local ParameterServerStrategy cluster (run by cli.launch from tests/test_ps_gpu.py): a small Keras
MLP trained with Model.train_step, so the trainer's backward goes through strategy.backward -> PSPushBucketer
(gradient buckets copied into the PS inboxes on the copy stream while backward runs) on GPU trainers with the shm
transport. Prints one JSON line per trainer: steps run, the PS global_step, and the final pulled parameters'
checksum (chief only)."""
import json
import os
import sys

import torch


def main():
    from distributed_tensorflow_amd import context
    from distributed_tensorflow_amd.keras import initializers, layers, losses, optimizers
    from distributed_tensorflow_amd.keras.models import Sequential
    from distributed_tensorflow_amd.parallel import TFConfigClusterResolver
    from distributed_tensorflow_amd.parallel.parameter_server import ParameterServerStrategy, run_parameter_server
    r = TFConfigClusterResolver()
    if r.is_ps:
        return run_parameter_server(r, device=context.default_device())
    steps = int(os.environ.get("PS_TEST_STEPS", "20"))
    dev = context.default_device()
    strat = ParameterServerStrategy(r, variable_partitioner="round_robin", device=dev)
    initializers.set_seed(5)
    with strat.scope():
        model = Sequential([layers.Dense(256, activation="relu"), layers.Dense(256, activation="relu"),
                            layers.Dense(10)])
        model.compile(optimizer=optimizers.SGD(0.05), loss=losses.SparseCategoricalCrossentropy(from_logits=True))
    g = torch.Generator().manual_seed(100 + strat.worker_index)
    for _ in range(steps):
        x = torch.randn(64, 128, generator=g).to(dev)
        y = torch.randint(0, 10, (64,), generator=g).to(dev)
        model.train_step((x, y))
    if dev.type == "cuda":
        torch.cuda.synchronize()
    strat.kv.add("test/finished", 1)
    strat.kv.wait_ge("test/finished", strat.num_workers, timeout_s=300)
    strat.pull()
    flat = strat._arena.flat.double()
    out = {"task": f"{r.task_type}{r.task_id}", "steps": steps, "global_step": strat.global_step(),
           "overlap_push": strat.overlap_push, "staleness": strat.staleness,
           "checksum": float((flat * torch.arange(1, flat.numel() + 1, device=flat.device, dtype=flat.dtype)
                              .remainder(977)).sum())}
    print("PSTEST " + json.dumps(out), flush=True)
    strat.shutdown()
    return 0


if __name__ == "__main__":
    sys.exit(main())
