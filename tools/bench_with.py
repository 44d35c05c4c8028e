"""Run bench.py with module attributes overridden or native switches set (A/B of switches that have no environment
variable):
    python tools/bench_with.py distributed_tensorflow_amd.ops.mha:_ATTN_DS=True -- --model bert_base --steps 20
    python tools/bench_with.py native:<dtf switch>=0 -- --model gpt2_medium"""
import importlib
import os
import runpy
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    argv = sys.argv[1:]
    cut = argv.index("--") if "--" in argv else len(argv)
    for spec in argv[:cut]:
        target, value = spec.split("=", 1)
        mod, attr = target.split(":")
        if mod == "native":
            from distributed_tensorflow_amd.ops._util import call
            call(attr, int(value))
            continue
        setattr(importlib.import_module(mod), attr, eval(value, {}))  # noqa: S307 - literals from the command line
    bench = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bench.py")
    sys.argv = [bench] + argv[cut + 1:]
    runpy.run_path(bench, run_name="__main__")


if __name__ == "__main__":
    main()
