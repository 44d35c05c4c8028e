"""Packaging: building the package compiles the native libraries first —
lib/libdtf_kernels.so (every csrc/kernels/*.hip, hipcc --offload-arch=gfx950) and
lib/libdtf_runtime.so (csrc/runtime/*.cc) — and ships them as package data.
``pip install .`` / ``python setup.py build`` therefore needs hipcc and g++ (no GPU)."""
import os
import sys

from setuptools import setup
from setuptools.command.build_py import build_py

ROOT = os.path.dirname(os.path.abspath(__file__))


class BuildNative(build_py):
    def run(self):
        sys.path.insert(0, ROOT)
        from distributed_tensorflow_amd import _build
        _build.build(verbose=True)
        super().run()


setup(cmdclass={"build_py": BuildNative})
