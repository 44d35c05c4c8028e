"""ctypes bindings to the in-tree native libraries.

The HIP kernel library is a plain C ABI (``extern "C"``) shared object: every
entry point takes raw device pointers, sizes and the ``hipStream_t`` of the
caller (PyTorch's current stream), so launches are capturable into a
hipGraph and ordered with the framework's own streams. Nothing here
falls back silently: on a machine with a GPU, a missing or stale library is an
error (``require_kernels``); CPU tensors take the reference (torch) path in
``ops`` explicitly.
"""
from __future__ import annotations

import ctypes
import os
import threading

_LIBDIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib")
_lock = threading.Lock()
_kern = None
_rt = None

P, I, L, F, U = ctypes.c_void_p, ctypes.c_int, ctypes.c_long, ctypes.c_float, ctypes.c_ulonglong

_KERNEL_SIGS = {
    "dtf_stream_create": [I],
    "dtf_gemm": [P, P, P, P, P, P, P, I, I, I, L, L, L, I, I, I, L, L, L, F, F, I, I, I, I, P, L, P],
    "dtf_conv_fwd": [P, P, P, P, P, P] + [I] * 15 + [I, I, I, P],
    "dtf_pwconv_fwd": [P, P, P, P, P, L, I, I, P],
    "dtf_conv_bn_apply_fwd": [P, P, P, P, P, P, P, P, L, I, I, I, P, P, P, P, P, F, F, P, P, P, P, P],
    "dtf_conv_dgrad": [P, P, P] + [I] * 15 + [I, F, I, P, L, P, P, P, P, P, P, P],
    "dtf_conv_dgrad_addsub2": [P, P, P, P, I, I, I, I, I, I, P, L, P, P, P, P, P, P],
    "dtf_conv_fwd_bn": [P, P, P, P] + [I] * 15 + [I, P, P, P, P, F, F, P, P, P, P, P, P],
    "dtf_conv_dgrad_x": [P, P, P] + [I] * 15 + [F, P, L, P, P, P, P, P, P, P, P, P, P],
    "dtf_bn_bwd_apply_coef": [P, P, P, L, I, P, P, P, P, P, P, P, P],
    "dtf_set_ew_variant": [I],
    "dtf_set_pw_dgrad": [I],
    "dtf_pw_conv_bwd": [P, P, P, P, P, I, P, P, P, P, P, P, L, L, I, I, P],
    "dtf_pw_conv_bwd_bn": [P, P, P, P, P, P, P, P, I, P, P, P, P, P, P, L, L, I, I, P, P, P, P, P, P],
    "dtf_bn_bwd_coef": [P, I, P, P, P, L, I, P, P, I, P, P],
    "dtf_set_pw_wgrad": [I],
    "dtf_set_c3_wgrad": [I],
    "dtf_set_split_penalty": [I],
    "dtf_set_ew_apply_nu": [I],
    "dtf_bn_bwd_partials": [P, P, P, P, P, P, L, I, P, P, P, P, I, P, I, P, P, P, P, P, P],
    "dtf_conv_wgrad": [P, P, P] + [I] * 15 + [I, I, I, P, L, P],
    "dtf_stem_wgrad": [P, P, P, I, I, I, I, P, L, P],
    "dtf_stem_wgrad_fused": [P, P, P, P, P, P, I, I, I, I, P, L, P],
    "dtf_bn_stats": [P, L, I, P, P, P],
    "dtf_bn_finalize": [P, I, P, P, P, P, L, I, F, F, P, P, P, P, P],
    "dtf_bn_infer_coeff": [P, P, P, P, I, F, P, P, P],
    "dtf_bn_apply": [P, P, P, P, P, L, I, I, P, P, P, P],
    "dtf_bn_bwd": [P, P, P, P, P, P, P, L, I, P, P, P, P, I, P, P, P, P, P, P],
    "dtf_layernorm_fwd": [P, P, P, P, P, P, L, I, F, P],
    "dtf_layernorm_bwd": [P, P, P, P, P, P, P, P, L, L, I, I, P],
    "dtf_layernorm_bwd2": [P, P, P, P, P, P, P, P, L, L, I, I, P, P],
    "dtf_add_dropout_layernorm_fwd": [P, P, P, P, P, P, P, P, L, I, F, F, U, P, P],
    "dtf_layernorm_bwd_part": [P, P, P, P, P, P, P, L, L, I, P, P, P, F, U, P, P],
    "dtf_maxpool_fwd": [P, P, P] + [I] * 12 + [P],
    "dtf_maxpool_bwd": [P, P, P] + [I] * 12 + [P],
    "dtf_add_dropout": [P, P, P, L, F, U, P, P],
    "dtf_softmax_ce_fwd": [P, I, P, P, P, L, I, F, P],
    "dtf_softmax_ce_bwd": [P, I, P, P, P, P, L, I, F, P],
    "dtf_nchw_to_s2d": [P, P, I, I, I, I, P],
    "dtf_stem_fwd": [P, P, P, P, P] + [I] * 9 + [P],
    "dtf_bn_relu_maxpool_fwd": [P, P, P, P, P] + [I] * 12 + [P],
    "dtf_maxpool_bn_bwd": [P, P, P, P, P, P] + [I] * 12 + [P, P, P, I, P, P],
    "dtf_gap_fwd": [P, P, I, I, I, I, P],
    "dtf_gap_bwd": [P, I, P, I, I, I, P],
    "dtf_optim_apply": [I, P, P, P, P, P, L, F, F, F, F, F, F, F, I, I, P, P, P, P],
    "dtf_sumsq": [P, L, P, I, P],
    "dtf_hp_ring_select": [P, I, I, P, P, P],
    "dtf_cast_f32_bf16": [P, P, L, P],
    "dtf_cast_bf16_f32": [P, P, L, P],
    "dtf_nchw_to_nhwc_pad": [P, P, I, I, I, I, P],
    "dtf_filter_to_crsk": [P, P, I, I, I, P],
    "dtf_filters_to_crsk": [P, I, I, P],
    "dtf_add_bf16": [P, P, P, L, F, F, P],
    "dtf_act": [P, P, P, L, I, I, P],
    "dtf_dropout": [P, P, L, F, U, P, P],
    "dtf_rng_advance": [P, P],
    "dtf_gemm256": [P, P, P, I, I, I, L, L, L, I, I, I, I, P, L, P],
    "dtf_gemm_w4": [P, P, P, I, I, I, L, L, L, I, I, I, I, P],
    "dtf_gemm_w4_var": [P, P, P, I, I, I, I, I, P],
    "dtf_gemm_w4_fp8": [P, P, P, I, I, I, L, L, L, I, I, I, P],
    "dtf_fp8_w4_enable": [I],
    "dtf_gemm_wgrad_bias": [P, P, P, P, I, I, I, L, L, L, F, P, L, P],
    "dtf_launch_counts": [P, I],
    # per-stream hipGraph executor (graph_sync.hip)
    "dtf_xs_epoch_inc": [P, I, P],
    "dtf_xs_signal": [P, I, P, I, P],
    "dtf_xs_wait": [P, I, P, I, P, I, P],
    "dtf_event_create": [],
    "dtf_event_destroy": [P],
    "dtf_event_record_external": [P, P],
    "dtf_stream_wait_external": [P, P],
    "dtf_gemm256_bn": [P, P, P, I, I, I, L, L, L, I, I, I, I, P],
    "dtf_gemm_dact": [P, P, P, P, I, I, I, I, L, L, L, I, I, P],
    "dtf_quant_fp8_exact": [P, P, L, P, P, P],
    "dtf_attn_fwd": [P, P, P, P, P, P, P, P, P, I, I, I, I, I, F, F, U, I, P, P],
    "dtf_attn_bwd": [P, P, P, P, P, P, P, P, P, P, P, P, P, P, I, I, I, I, I, F, F, U, I, P, P],
    "dtf_attn_bwd_ds": [P, P, P, P, P, P, P, P, P, P, P, P, P, P, I, I, I, I, I, F, F, U, I, P, P, P],
    "dtf_colsum": [P, L, I, P, I, P, L, P],
    "dtf_embed_fwd": [P, P, P, P, P, P, P, L, I, I, P],
    "dtf_embed_bwd_sorted": [P, P, P, P, L, I, P],
    "dtf_sort_keys": [P, L, I, P, P, P, L, P],
    "dtf_gather_rows": [P, P, P, L, I, P],
    "dtf_gather_cols": [P, I, L, L, P, L, P, P],
    "dtf_gather_rows_bwd": [P, P, P, L, P, L, I, P],
    "dtf_embed_bwd_small": [P, P, P, L, I, I, I, P, L, P],
    "dtf_softmax_ce": [P, I, P, P, P, I, L, I, F, F, P],
    "dtf_softmax_fwd": [P, P, L, I, I, F, I, P, P],
    "dtf_softmax_bwd": [P, P, P, L, I, F, P],
    "dtf_gemm_fp8": [P, P, P, P, P, P, I, I, I, L, L, L, I, I, P],
    "dtf_quant_fp8": [P, P, L, P, P, I, P],
    "dtf_fp8_update_scale": [P, P, F, P],
    "dtf_quant_fp8_t": [P, P, I, P, P, P, P, P, I, I, I, I, P, P, P],
    "dtf_fp8_update_scale2": [P, P, P, F, F, P],
    "dtf_reduce_rows": [P, L, I, L, P, I, P],
    "dtf_gemm_fp8_ex": [P, P, P, P, P, P, I, I, I, L, L, L, I, I, I, F, I, P, L, P, P],
    "dtf_gemm_fp8_q8": [P, P, P, P, P, P, I, I, I, L, L, I, I, P, I, P, P, P, P, I, P, P, P, P, P, P],
    "dtf_quant_fp8_t2": [P, P, I, P, P, P, P, P, I, I, I, I, P, P, P, P, P, P],
    "dtf_group_rows_once": [P, L, I, L, I, P, P],
    "dtf_sum_rows": [P, L, I, L, P, I, P],  # void: the int return value is meaningless
    "dtf_ipc_export": [P, P, P],
    "dtf_ipc_open": [P, P],
    "dtf_ipc_close": [P],
    "dtf_p2p_allreduce_f32": [P, P, P, P, P, L, I, I, I, I, I, P, P],
    "dtf_memcpy_async": [P, P, L, P],
}


_RESTYPES = {"dtf_stream_create": P, "dtf_event_create": P}


class NativeMissing(RuntimeError):
    pass


def _load(path):
    # torch must be imported first so its HIP runtime (same soname) is the one bound.
    import torch  # noqa: F401
    return ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)


def kernels_available() -> bool:
    return os.path.exists(os.path.join(_LIBDIR, "libdtf_kernels.so"))


def kernels():
    """Return the loaded kernel library (raises NativeMissing if it is not built)."""
    global _kern
    if _kern is not None:
        return _kern
    with _lock:
        if _kern is not None:
            return _kern
        path = os.path.join(_LIBDIR, "libdtf_kernels.so")
        if not os.path.exists(path):
            raise NativeMissing(
                f"{path} is missing: run `python -m distributed_tensorflow_amd._build` (hipcc, gfx950)")
        lib = _load(path)
        for name, sig in _KERNEL_SIGS.items():
            fn = getattr(lib, name, None)
            if fn is None:
                continue
            fn.argtypes = sig
            fn.restype = _RESTYPES.get(name, ctypes.c_int)
        _kern = lib
        return lib


def runtime():
    """Return the host C++ runtime library (checkpoint IO, KV store, PS transport...)."""
    global _rt
    if _rt is not None:
        return _rt
    with _lock:
        if _rt is not None:
            return _rt
        path = os.path.join(_LIBDIR, "libdtf_runtime.so")
        if not os.path.exists(path):
            from . import _build
            _build.build_runtime(verbose=False)
        lib = ctypes.CDLL(path)
        from . import _runtime_sigs
        _runtime_sigs.declare(lib)
        _rt = lib
        return lib


def call(name, *args):
    """Invoke a kernel entry point; raise on a non-zero status."""
    fn = getattr(kernels(), name)
    rc = fn(*args)
    if rc != 0:
        raise RuntimeError(f"{name} failed with status {rc}")
    return rc
