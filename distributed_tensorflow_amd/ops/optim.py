"""Fused optimizer apply (csrc/kernels/optim.hip) over flat f32 arenas."""
from __future__ import annotations

from ._util import call, ptr, step_abort_ptr, stream

KINDS = {"sgd": 0, "adam": 1, "adagrad": 2, "adadelta": 3, "ftrl": 4, "rmsprop": 5, "lamb": 6}


def optim_apply(kind, p, g, s1, s2, p16, hp, *, b1=0.9, b2=0.999, eps=1e-8, wd=0.0, mom=0.0, l1=0.0, l2=0.0,
                nesterov=False, zero_grad=False, sumsq=None):
    """One streaming launch: update p (and slots s1/s2), write the bf16 copy p16, optionally zero g. Inside a
    per-stream hipGraph capture the kernel also reads the capture's error flag and applies nothing once a
    cross-stream wait of the step timed out (graph_sync.hip)."""
    k = KINDS[kind] if isinstance(kind, str) else int(kind)
    call("dtf_optim_apply", k, ptr(p), ptr(g), ptr(s1), ptr(s2), ptr(p16), p.numel(), float(b1), float(b2),
         float(eps), float(wd), float(mom), float(l1), float(l2), int(nesterov), int(zero_grad), ptr(hp), ptr(sumsq),
         step_abort_ptr(), stream())


def sumsq(x, out, zero=True):
    call("dtf_sumsq", ptr(x), x.numel(), ptr(out), int(zero), stream())
