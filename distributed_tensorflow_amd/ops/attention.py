"""Scaled dot-product attention.

GPU: scores = Q K^T on the batched MFMA GEMM, masked/causal softmax kernel, P V on the GEMM
(K3 + K7 composition); every piece has a hand-written backward. CPU: f32 reference.
Layout: q, k, v are [B, H, S, D] (bf16 on GPU).
"""
from __future__ import annotations

import math

import torch

from ._util import BF16, on_gpu
from .linalg import bmm
from .nn import softmax


def attention(q, k, v, causal=False, mask=None, scale=None, dropout=0.0, training=False):
    """mask: optional additive f32 mask broadcastable as [B, 1, 1, Sk] (0 keep, -inf/-1e4 drop)."""
    B, H, Sq, D = q.shape
    Sk = k.shape[2]
    scale = scale if scale is not None else 1.0 / math.sqrt(D)
    if on_gpu(q):
        q3 = q.reshape(B * H, Sq, D)
        k3 = k.reshape(B * H, Sk, D)
        v3 = v.reshape(B * H, Sk, D)
        s = bmm(q3, k3, transpose_b=True)  # [BH, Sq, Sk] bf16
        am = None
        if mask is not None:
            am = mask.reshape(B, Sk).float().repeat_interleave(H, 0).contiguous()
        p = softmax(s.reshape(B * H, Sq, Sk), scale=scale, causal=causal, add_mask=am)
        if dropout and training:
            from .nn import dropout as _drop
            p = _drop(p, dropout)
        o = bmm(p, v3)
        return o.reshape(B, H, Sq, D)
    s = torch.matmul(q.float(), k.float().transpose(-1, -2)) * scale
    if causal:
        m = torch.ones(Sq, Sk, dtype=torch.bool, device=q.device).tril(Sk - Sq)
        s = s.masked_fill(~m, float("-inf"))
    if mask is not None:
        s = s + mask.reshape(B, 1, 1, Sk).float()
    p = torch.softmax(s, -1)
    if dropout and training:
        p = torch.nn.functional.dropout(p, dropout)
    return torch.matmul(p, v.float()).to(q.dtype)


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


del BF16
