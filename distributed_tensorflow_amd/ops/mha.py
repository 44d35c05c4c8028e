"""Scaled dot-product attention.

GPU: one fused HIP kernel per direction (csrc/kernels/attention.hip): online-softmax forward that never
materialises the [S, S] scores, and a deterministic two-kernel backward (dK/dV by key blocks, dQ by
query blocks), with causal and additive key masks and in-kernel dropout on the probabilities. The
packed entry point reads Q/K/V straight out of the fused QKV projection [B, S, 3*H*64] and writes
O as [B, S, H*64], so no head split/merge copies exist; its backward writes one packed dQKV.
Head dims other than 64 use the composed path (MFMA batched GEMM + softmax kernel). CPU: f32 reference.
"""
from __future__ import annotations

import ctypes
import math

import torch

from ._util import BF16, F32, call, on_gpu, ptr, rng_counter, stream
from .linalg import bmm
from .nn import softmax

_seed_counter = [0]

# Backward through a dS^T scratch (dtf_attn_bwd_ds: the dK/dV kernel stores dS, dQ is a memory-bound GEMM over it)
# instead of a dQ kernel that recomputes the scores, probabilities and dP: causal attention only (None; tests set True /
# False to force a path) — measured (tools/bench_attention.py, profiles/r4_attention_bench.txt): GPT-2-medium causal S=1024
# 178 -> 158 us (213 -> 183 with dropout); BERT-base S=512 203 -> 227 us (the dS round trip costs more than the
# recompute saves when no tiles are skipped)
_ATTN_DS = None
# The dS^T scratch is O(B*H*S^2) (GPT-2-medium S=1024 B=8: 268 MB per call); above this many bytes the backward takes
# the O(S) recompute kernel instead, so a long-context run keeps flash attention's memory bound.
DS_SCRATCH_MAX_BYTES = 1 << 30


def ds_scratch_bytes(B, H, Sq, Sk):
    return 2 * B * H * Sk * (-(-Sq // 64) * 64)


def uses_ds_path(causal, B, H, Sq, Sk):
    """True when the attention backward goes through the dS^T scratch (dtf_attn_bwd_ds)."""
    if not (_ATTN_DS or (_ATTN_DS is None and causal)):
        return False
    return ds_scratch_bytes(B, H, Sq, Sk) <= DS_SCRATCH_MAX_BYTES


def _bwd(args_before_ds, B, H, Sq, Sk, dev):
    """Run the attention backward (args: the dtf_attn_bwd argument list, causal flag at [-3])."""
    causal = bool(args_before_ds[-3])
    if uses_ds_path(causal, B, H, Sq, Sk):
        ds = torch.empty(B * H * Sk * (-(-Sq // 64) * 64), dtype=BF16, device=dev)
        call("dtf_attn_bwd_ds", *args_before_ds[:-1], ptr(ds), args_before_ds[-1])
    else:
        call("dtf_attn_bwd", *args_before_ds)


def _next_seed(seed, device):
    """(host seed, device step-counter pointer or None): see ops.nn._auto_seed."""
    if seed is not None:
        return seed, None
    _seed_counter[0] += 1
    return (_seed_counter[0] * 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF, rng_counter(device)


def _strides3(b, s, h):
    arr = (ctypes.c_long * 3)(int(b), int(s), int(h))
    return arr, ctypes.addressof(arr)


class _FlashPackedFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, kmask, heads, causal, scale, dropout, seed, ctr):
        qkv = qkv.contiguous()
        B, S, T = qkv.shape
        D = T // (3 * heads)
        HD = heads * D
        o = torch.empty(B, S, HD, dtype=BF16, device=qkv.device)
        lse = torch.empty(B * heads, S, dtype=F32, device=qkv.device)
        qs, qsp = _strides3(S * T, T, D)
        os_, osp = _strides3(S * HD, HD, D)
        base = qkv.data_ptr()
        call("dtf_attn_fwd", base, base + 2 * HD, base + 4 * HD, qsp, qsp, ptr(o), osp, ptr(lse), ptr(kmask), B, heads, S,
             S, D, float(scale), float(dropout), seed, int(causal), ctr, stream())
        ctx.save_for_backward(qkv, o, lse, kmask)
        ctx.cfg = (heads, causal, scale, dropout, seed, ctr)
        return o

    @staticmethod
    def backward(ctx, do):
        qkv, o, lse, kmask = ctx.saved_tensors
        heads, causal, scale, dropout, seed, ctr = ctx.cfg
        do = do.to(BF16).contiguous()
        B, S, T = qkv.shape
        D = T // (3 * heads)
        HD = heads * D
        dqkv = torch.empty_like(qkv)
        dvec = torch.empty(B * heads, S, dtype=F32, device=qkv.device)
        qs, qsp = _strides3(S * T, T, D)
        os_, osp = _strides3(S * HD, HD, D)
        base, gb = qkv.data_ptr(), dqkv.data_ptr()
        _bwd((base, base + 2 * HD, base + 4 * HD, qsp, qsp, ptr(o), ptr(do), osp, ptr(lse), ptr(dvec),
              gb, gb + 2 * HD, gb + 4 * HD, ptr(kmask), B, heads, S, S, D, float(scale), float(dropout), seed,
              int(causal), ctr, stream()), B, heads, S, S, qkv.device)
        return dqkv, None, None, None, None, None, None, None


class _FlashFn(torch.autograd.Function):
    """Separate q, k, v tensors in [B, H, S, D] layout."""

    @staticmethod
    def forward(ctx, q, k, v, kmask, causal, scale, dropout, seed, ctr):
        q, k, v = q.contiguous(), k.contiguous(), v.contiguous()
        B, H, Sq, D = q.shape
        Sk = k.shape[2]
        o = torch.empty_like(q)
        lse = torch.empty(B * H, Sq, dtype=F32, device=q.device)
        qs, qsp = _strides3(H * Sq * D, D, Sq * D)
        ks, ksp = _strides3(H * Sk * D, D, Sk * D)
        call("dtf_attn_fwd", ptr(q), ptr(k), ptr(v), qsp, ksp, ptr(o), qsp, ptr(lse), ptr(kmask), B, H, Sq, Sk, D,
             float(scale), float(dropout), seed, int(causal), ctr, stream())
        ctx.save_for_backward(q, k, v, o, lse, kmask)
        ctx.cfg = (causal, scale, dropout, seed, ctr)
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v, o, lse, kmask = ctx.saved_tensors
        causal, scale, dropout, seed, ctr = ctx.cfg
        do = do.to(BF16).contiguous()
        B, H, Sq, D = q.shape
        Sk = k.shape[2]
        dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
        dvec = torch.empty(B * H, Sq, dtype=F32, device=q.device)
        qs, qsp = _strides3(H * Sq * D, D, Sq * D)
        ks, ksp = _strides3(H * Sk * D, D, Sk * D)
        _bwd((ptr(q), ptr(k), ptr(v), qsp, ksp, ptr(o), ptr(do), qsp, ptr(lse), ptr(dvec), ptr(dq),
              ptr(dk), ptr(dv), ptr(kmask), B, H, Sq, Sk, D, float(scale), float(dropout), seed, int(causal),
              ctr, stream()), B, H, Sq, Sk, q.device)
        return dq, dk, dv, None, None, None, None, None, None


def _kmask(mask, B, Sk):
    if mask is None:
        return None
    return mask.reshape(B, Sk).float().contiguous()


def attention(q, k, v, causal=False, mask=None, scale=None, dropout=0.0, training=False, seed=None):
    """q, k, v: [B, H, S, D]. mask: optional additive f32 mask broadcastable as [B, 1, 1, Sk]."""
    B, H, Sq, D = q.shape
    Sk = k.shape[2]
    scale = scale if scale is not None else 1.0 / math.sqrt(D)
    rate = float(dropout) if (dropout and training) else 0.0
    if on_gpu(q):
        if D == 64 and k.shape[2] == v.shape[2]:
            seed, ctr = _next_seed(seed, q.device)
            return _FlashFn.apply(q.to(BF16), k.to(BF16), v.to(BF16), _kmask(mask, B, Sk), bool(causal),
                                  float(scale), rate, seed, ctr)
        return _composed(q, k, v, causal, mask, scale, rate)
    s = torch.matmul(q.float(), k.float().transpose(-1, -2)) * scale
    if causal:
        m = torch.ones(Sq, Sk, dtype=torch.bool, device=q.device).tril(Sk - Sq)
        s = s.masked_fill(~m, float("-inf"))
    if mask is not None:
        s = s + mask.reshape(B, 1, 1, Sk).float()
    p = torch.softmax(s, -1)
    if rate:
        p = torch.nn.functional.dropout(p, rate)
    return torch.matmul(p, v.float()).to(q.dtype)


def attention_packed(qkv, heads, causal=False, mask=None, scale=None, dropout=0.0, training=False, seed=None):
    """Self-attention on the fused projection output qkv [B, S, 3*H*D] -> [B, S, H*D]."""
    B, S, T = qkv.shape
    D = T // (3 * heads)
    scale = scale if scale is not None else 1.0 / math.sqrt(D)
    rate = float(dropout) if (dropout and training) else 0.0
    if on_gpu(qkv) and D == 64 and qkv.dtype == BF16:
        seed, ctr = _next_seed(seed, qkv.device)
        return _FlashPackedFn.apply(qkv, _kmask(mask, B, S), heads, bool(causal), float(scale), rate, seed, ctr)
    q, k, v = split_qkv(qkv, heads)
    return merge_heads(attention(q, k, v, causal, mask, scale, dropout, training))


def _composed(q, k, v, causal, mask, scale, rate):
    """K3 + K7 composition (batched MFMA GEMMs around the masked softmax kernel)."""
    B, H, Sq, D = q.shape
    Sk = k.shape[2]
    q3 = q.reshape(B * H, Sq, D)
    k3 = k.reshape(B * H, Sk, D)
    v3 = v.reshape(B * H, Sk, D)
    s = bmm(q3, k3, transpose_b=True)
    am = None
    if mask is not None:
        am = mask.reshape(B, Sk).float().repeat_interleave(H, 0).contiguous()
    p = softmax(s.reshape(B * H, Sq, Sk), scale=scale, causal=causal, add_mask=am)
    if rate:
        from .nn import dropout as _drop
        p = _drop(p, rate)
    return bmm(p, v3).reshape(B, H, Sq, D)


def reference_attention(q, k, v, causal=False, mask=None, scale=None, keep_mask=None, keep=1.0):
    """f32 reference with an explicit dropout keep-mask (tests)."""
    B, H, Sq, D = q.shape
    Sk = k.shape[2]
    scale = scale if scale is not None else 1.0 / math.sqrt(D)
    s = torch.matmul(q.float(), k.float().transpose(-1, -2)) * scale
    if causal:
        m = torch.ones(Sq, Sk, dtype=torch.bool, device=q.device).tril(Sk - Sq)
        s = s.masked_fill(~m, float("-inf"))
    if mask is not None:
        s = s + mask.reshape(B, 1, 1, Sk).float()
    p = torch.softmax(s, -1)
    if keep_mask is not None:
        p = p * keep_mask / keep
    return torch.matmul(p, v.float())


def split_heads(x, heads):
    """[B, S, H*D] -> [B, H, S, D] (contiguous)."""
    B, S, HD = x.shape
    return x.reshape(B, S, heads, HD // heads).permute(0, 2, 1, 3).contiguous()


def merge_heads(x):
    B, H, S, D = x.shape
    return x.permute(0, 2, 1, 3).reshape(B, S, H * D).contiguous()


def split_qkv(qkv, heads):
    """[B, S, 3*H*D] -> three [B, H, S, D] tensors."""
    B, S, T = qkv.shape
    D = T // (3 * heads)
    x = qkv.reshape(B, S, 3, heads, D).permute(2, 0, 3, 1, 4).contiguous()
    return x[0], x[1], x[2]
