"""Small helpers shared by the op wrappers."""
from __future__ import annotations

import torch

from .. import _native

BF16 = torch.bfloat16
F32 = torch.float32


def ptr(t):
    """Raw device pointer of a tensor (None -> NULL)."""
    if t is None:
        return None
    return t.data_ptr()


def stream():
    return torch.cuda.current_stream().cuda_stream


def on_gpu(*ts) -> bool:
    for t in ts:
        if t is not None and isinstance(t, torch.Tensor):
            return t.is_cuda
    return False


def K():
    """The kernel library; raises loudly when it is absent (no silent eager fallback on GPU)."""
    return _native.kernels()


def call(name, *args):
    fn = getattr(K(), name)
    rc = fn(*args)
    if rc != 0:
        raise RuntimeError(f"{name} failed with status {rc}")


def contig(t):
    return t if t is None or t.is_contiguous() else t.contiguous()


def bf16_shadow(param):
    """bf16 compute copy of an f32 master variable (kept fresh by the fused optimizer)."""
    s = getattr(param, "_dtf_bf16", None)
    ver = getattr(param, "_dtf_version", None)
    cur = param._version
    if s is None:
        s = param.detach().to(BF16)
        try:
            param._dtf_bf16 = s
        except AttributeError:
            pass
        param._dtf_version = cur
        param._dtf_bf16_owned = True
        return s
    if getattr(param, "_dtf_bf16_owned", False) and ver != cur:
        s.copy_(param.detach())
        param._dtf_version = cur
    return s


class _WeightsEpoch:
    """Bumped by every fused optimizer step: derived weight layouts (e.g. the
    CRSK filter copy used by conv data-gradients) are refreshed lazily."""
    value = 0


def bump_weights_epoch():
    _WeightsEpoch.value += 1


def weights_epoch():
    return _WeightsEpoch.value


def crsk_shadow(param, K, RS, C):
    """bf16 [C][R][S][K] copy of a KRSC filter for the dgrad implicit GEMM."""
    key = (weights_epoch(), param._version)
    s = getattr(param, "_dtf_crsk", None)
    if s is not None and getattr(param, "_dtf_crsk_key", None) == key:
        return s
    w16 = bf16_shadow(param)
    if s is None:
        s = torch.empty((C, RS, K), dtype=BF16, device=param.device)
        param._dtf_crsk = s
    call("dtf_filter_to_crsk", ptr(w16), ptr(s), K, RS, C, stream())
    param._dtf_crsk_key = key
    return s
