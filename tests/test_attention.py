"""Fused attention kernel (csrc/kernels/attention.hip) vs an f32 PyTorch reference.

Covers: non-causal / causal, ragged S (not a multiple of the 64-row tiles), additive key-padding masks,
the packed-QKV entry point, and in-kernel dropout (the keep-mask is regenerated on the host from the
same counter hash and fed to the reference).
"""
import math

import numpy as np
import pytest
import torch

from distributed_tensorflow_amd import ops
import importlib

A = importlib.import_module("distributed_tensorflow_amd.ops.mha")

BF = torch.bfloat16


def close(a, b, tol):
    a, b = a.float(), b.float()
    err = (a - b).abs().max().item()
    ref = b.abs().max().item() + 1e-6
    assert err <= tol * ref, f"max err {err} vs ref scale {ref} (tol {tol})"


def _fmix32(h):
    h = h ^ (h >> np.uint32(16))
    h = h * np.uint32(0x85EBCA6B)
    h = h ^ (h >> np.uint32(13))
    h = h * np.uint32(0xC2B2AE35)
    h = h ^ (h >> np.uint32(16))
    return h


def keep_mask(seed, B, H, Sq, Sk, keep):
    """Host replica of the kernel's dropout hash: returns (keep-mask [B,H,Sq,Sk], realised keep prob)."""
    thr = int(np.clip(np.rint(np.float32(keep) * np.float32(65536.0)), 1, 65536))
    s32 = np.uint32((seed ^ (seed >> 32)) & 0xFFFFFFFF)
    nkq = (Sk + 3) // 4
    with np.errstate(over="ignore"):
        bh = np.arange(B * H, dtype=np.uint32)[:, None, None]
        q = np.arange(Sq, dtype=np.uint32)[None, :, None]
        k = np.arange(Sk, dtype=np.uint32)[None, None, :]
        salt = _fmix32(s32 ^ (bh * np.uint32(0x9E3779B9)))
        x = _fmix32((q * np.uint32(nkq) + (k >> np.uint32(2))) ^ salt)
        y = (x ^ (x >> np.uint32(16))) * np.uint32(0x45D9F3B)
        j = k & np.uint32(3)
        w = np.where(j < 2, x, y)
        u = (w >> (np.uint32(16) * (j & np.uint32(1)))) & np.uint32(0xFFFF)
    m = (u < thr).reshape(B, H, Sq, Sk).astype(np.float32)
    return torch.from_numpy(m), thr / 65536.0


def test_ds_scratch_route_is_capped():
    """The causal backward's dS^T scratch is O(S^2): GPT-2-medium S=1024 keeps it, a long context takes the O(S)
    recompute kernel (an unbounded scratch could OOM a long-context run)."""
    if A._ATTN_DS is False:
        pytest.skip("DTF_ATTN_DS=0")
    assert A.uses_ds_path(True, 8, 16, 1024, 1024)
    assert A.ds_scratch_bytes(8, 16, 8192, 8192) > A.DS_SCRATCH_MAX_BYTES
    assert not A.uses_ds_path(True, 8, 16, 8192, 8192)


def test_cpu_reference_paths():
    q, k, v = (torch.randn(2, 3, 16, 8) for _ in range(3))
    o = ops.attention(q, k, v, causal=True)
    r = A.reference_attention(q, k, v, causal=True)
    close(o, r, 1e-5)
    qkv = torch.randn(2, 16, 3 * 3 * 8)
    o2 = ops.attention_packed(qkv, 3)
    qq, kk, vv = A.split_qkv(qkv, 3)
    close(o2, A.merge_heads(A.reference_attention(qq, kk, vv)), 1e-5)
    m, keff = keep_mask(12345, 1, 2, 4, 5, 0.9)
    assert m.shape == (1, 2, 4, 5) and abs(keff - 0.9) < 1e-4


def _run(cuda, B, H, Sq, Sk, causal, masked, dropout=0.0, seed=7):
    torch.manual_seed(0)
    q = torch.randn(B, H, Sq, 64, device=cuda).to(BF).requires_grad_(True)
    k = torch.randn(B, H, Sk, 64, device=cuda).to(BF).requires_grad_(True)
    v = torch.randn(B, H, Sk, 64, device=cuda).to(BF).requires_grad_(True)
    mask = None
    if masked:
        lens = torch.randint(Sk // 2, Sk + 1, (B,))
        mask = torch.zeros(B, Sk, device=cuda)
        for b in range(B):
            mask[b, lens[b]:] = -10000.0
    o = ops.attention(q, k, v, causal=causal, mask=mask, dropout=dropout, training=dropout > 0, seed=seed)
    km, keff = keep_mask(seed, B, H, Sq, Sk, 1 - dropout) if dropout else (None, 1.0)
    km = km.to(cuda) if km is not None else None
    qr, kr, vr = (t.detach().float().requires_grad_(True) for t in (q, k, v))
    r = A.reference_attention(qr, kr, vr, causal=causal, mask=mask, keep_mask=km, keep=keff)
    close(o, r, 2e-2)
    do = torch.randn_like(r)
    r.backward(do)
    o.backward(do.to(BF))
    close(q.grad, qr.grad, 3e-2)
    close(k.grad, kr.grad, 3e-2)
    close(v.grad, vr.grad, 3e-2)


@pytest.mark.gpu
@pytest.mark.parametrize("B,H,Sq,Sk,causal,masked", [
    (2, 3, 128, 128, False, False),
    (2, 2, 200, 200, False, True),
    (1, 4, 256, 256, True, False),
    (2, 2, 100, 164, True, False),
    (3, 2, 64, 512, False, True),
])
def test_flash_attention(cuda, B, H, Sq, Sk, causal, masked):
    _run(cuda, B, H, Sq, Sk, causal, masked)


@pytest.mark.gpu
def test_flash_attention_dropout(cuda):
    _run(cuda, 2, 2, 128, 192, False, True, dropout=0.1, seed=99)
    _run(cuda, 1, 2, 256, 256, True, False, dropout=0.2, seed=2**40 + 3)


@pytest.mark.gpu
def test_flash_attention_packed(cuda):
    B, S, H = 2, 192, 4
    qkv = (torch.randn(B, S, 3 * H * 64, device=cuda) * 0.5).to(BF).requires_grad_(True)
    mask = torch.zeros(B, S, device=cuda)
    mask[1, 150:] = -10000.0
    o = ops.attention_packed(qkv, H, causal=False, mask=mask)
    qr = qkv.detach().float().requires_grad_(True)
    q, k, v = A.split_qkv(qr, H)
    r = A.merge_heads(A.reference_attention(q, k, v, mask=mask))
    close(o, r, 2e-2)
    do = torch.randn_like(r)
    r.backward(do)
    o.backward(do.to(BF))
    close(qkv.grad, qr.grad, 3e-2)


@pytest.mark.gpu
@pytest.mark.parametrize("B,H,Sq,Sk,causal,masked,dropout", [
    (2, 3, 128, 128, False, False, 0.0),
    (2, 2, 200, 200, False, True, 0.0),
    (1, 4, 256, 256, True, False, 0.0),
    (2, 2, 100, 164, True, False, 0.0),
    (3, 2, 64, 512, False, True, 0.0),
    (2, 2, 128, 192, False, True, 0.1),
    (1, 2, 256, 256, True, False, 0.2),
])
def test_flash_attention_ds_backward(cuda, monkeypatch, B, H, Sq, Sk, causal, masked, dropout):
    """The dS^T-scratch backward (dtf_attn_bwd_ds: dK/dV kernel stores dS, dQ is a GEMM over it) against the f32
    reference, on the shapes of the recompute backward's tests (ragged lengths, causal with Sk > Sq, dropout)."""
    monkeypatch.setattr(A, "_ATTN_DS", True)
    _run(cuda, B, H, Sq, Sk, causal, masked, dropout=dropout, seed=99 if dropout else 7)


@pytest.mark.gpu
def test_flash_attention_ds_packed_matches_recompute(cuda, monkeypatch):
    """Packed QKV with causal masking and dropout: the dS^T path and the recompute path agree up to f32 summation
    order (D = rowsum(dO * O) is summed by another kernel, dQ by a GEMM over the bf16 dS both paths use)."""
    B, S, H = 2, 320, 4
    torch.manual_seed(1)
    qkv = (torch.randn(B, S, 3 * H * 64, device=cuda) * 0.5).to(BF)
    do = torch.randn(B, S, H * 64, device=cuda).to(BF)
    grads = []
    for ds in (False, True):
        monkeypatch.setattr(A, "_ATTN_DS", ds)
        x = qkv.clone().requires_grad_(True)
        o = ops.attention_packed(x, H, causal=True, dropout=0.1, training=True, seed=5)
        (g,) = torch.autograd.grad(o, [x], do)
        grads.append(g.float().reshape(B, S, 3, H * 64))
    a, b = grads
    for j in range(3):
        assert (a[:, :, j] - b[:, :, j]).abs().max().item() <= 1e-2 * a[:, :, j].abs().max().item(), j
