"""Build the native libraries in-tree.

* ``lib/libdtf_kernels.so`` — every ``csrc/kernels/*.hip`` compiled with
  ``hipcc --offload-arch=gfx950`` (CDNA4 code objects only; no other targets,
  no hipify, no CUDA shims).
* ``lib/libdtf_runtime.so`` — the host-side C++ runtime (``csrc/runtime/*.cc``):
  tensor-bundle checkpoint IO, TFRecord/event writer, CRC32C, the TCP
  rendezvous / KV store, the parameter-server transport and the CPU
  shared-memory all-reduce, and the RCCL communicator (librccl bound at run time).

The reference has no native code of its own; these are the
MI355X-native equivalents of the TF runtime pieces it relies on.

Objects are rebuilt only when a source or header is newer than the object,
so ``build()`` is cheap when nothing changed. Run ``python -m
distributed_tensorflow_amd._build`` to build by hand.
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "csrc")
LIBDIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib")
OBJDIR = os.path.join(ROOT, "build", "obj")
ARCH = os.environ.get("DTF_OFFLOAD_ARCH", "gfx950")

KERNELS_SO = os.path.join(LIBDIR, "libdtf_kernels.so")
RUNTIME_SO = os.path.join(LIBDIR, "libdtf_runtime.so")


def _hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found: the gfx950 kernels cannot be built")


def _newest(paths):
    return max((os.path.getmtime(p) for p in paths if os.path.exists(p)), default=0.0)


def _sources(sub, exts):
    d = os.path.join(CSRC, sub)
    if not os.path.isdir(d):
        return [], []
    srcs = sorted(os.path.join(d, f) for f in os.listdir(d) if f.endswith(exts))
    hdrs = sorted(os.path.join(d, f) for f in os.listdir(d) if f.endswith((".h", ".hpp")))
    return srcs, hdrs


def _compile(cmd, src, obj, deps, verbose):
    if os.path.exists(obj) and os.path.getmtime(obj) >= _newest([src] + deps):
        return obj
    os.makedirs(os.path.dirname(obj), exist_ok=True)
    if verbose:
        print("[dtf-build]", os.path.relpath(src, ROOT), flush=True)
    r = subprocess.run(cmd + ["-c", src, "-o", obj + ".tmp"], capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {src}\n{r.stdout}\n{r.stderr}")
    os.replace(obj + ".tmp", obj)
    return obj


def _link(cmd, objs, out, verbose):
    # the object list is part of the staleness check: a removed source must relink too
    manifest = os.path.join(OBJDIR, os.path.basename(out) + ".objs")
    listing = "\n".join(sorted(os.path.basename(o) for o in objs))
    same = os.path.exists(manifest) and open(manifest).read() == listing
    if same and os.path.exists(out) and os.path.getmtime(out) >= _newest(objs):
        return out
    os.makedirs(os.path.dirname(out), exist_ok=True)
    if verbose:
        print("[dtf-build] link", os.path.relpath(out, ROOT), flush=True)
    r = subprocess.run(cmd + objs + ["-o", out + ".tmp"], capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed: {out}\n{r.stdout}\n{r.stderr}")
    os.replace(out + ".tmp", out)
    with open(manifest, "w") as f:
        f.write(listing)
    return out


def build_kernels(verbose=True, jobs=None):
    srcs, hdrs = _sources("kernels", (".hip",))
    hipcc = _hipcc()
    flags = [hipcc, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-Wno-unused-result",
             "-munsafe-fp-atomics", "-mcode-object-version=5"]
    jobs = jobs or min(8, os.cpu_count() or 4, int(os.environ.get("MAX_JOBS", "8")))
    with cf.ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(lambda s: _compile(flags, s, os.path.join(OBJDIR, "kernels",
                                                                     os.path.basename(s) + ".o"), hdrs, verbose),
                           srcs))
    so = _link([hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC"], objs, KERNELS_SO, verbose)
    # a declaration in the wrong namespace links fine into a shared library and fails only at dlopen on the GPU box:
    # refuse undefined C++ symbols of our own here
    r = subprocess.run(["nm", "-u", "-C", so], capture_output=True, text=True)
    bad = [ln.strip() for ln in r.stdout.splitlines() if "dtf" in ln or "GemmArgs" in ln]
    if bad:
        raise RuntimeError(f"{so}: undefined symbols of our own: {bad[:8]}")
    return so


def build_runtime(verbose=True, jobs=None):
    srcs, hdrs = _sources("runtime", (".cc", ".cpp"))
    srcs = [s for s in srcs if not os.path.basename(s).startswith("selftest")]  # sanitizer driver (tools/)
    if not srcs:
        return None
    cxx = os.environ.get("CXX", "g++")
    flags = [cxx, "-O2", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-function", "-pthread"]
    jobs = jobs or min(8, os.cpu_count() or 4)
    with cf.ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(lambda s: _compile(flags, s, os.path.join(OBJDIR, "runtime",
                                                                     os.path.basename(s) + ".o"), hdrs, verbose),
                           srcs))
    return _link([cxx, "-shared", "-fPIC", "-pthread", "-ldl"], objs, RUNTIME_SO, verbose)


def build(verbose=True):
    rt = build_runtime(verbose)
    k = build_kernels(verbose)
    return k, rt


if __name__ == "__main__":
    build(verbose="-q" not in sys.argv)
