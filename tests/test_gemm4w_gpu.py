"""The 4-wave 256x256 GEMM (gemm4w.hip: 128x128 output per wave, LDS-DMA staged halves, one barrier per K-tile)
against an f32 PyTorch reference of the same bf16 operands in all four operand layouts (K-contiguous / K-outer A and
B), bf16 and f32 outputs, ragged M / N edges; and its fp8 forms (e4m3 x e4m3, e5m2 x e4m3 block-scaled MFMA) against
the same fp8 bytes decoded to f32."""
import pytest
import torch

from distributed_tensorflow_amd.ops._util import call, ptr, stream

pytestmark = pytest.mark.gpu
BF = torch.bfloat16


def _close(a, b, tol):
    err = (a.float() - b.float()).abs().max().item()
    ref = b.float().abs().max().item() + 1e-6
    assert err <= tol * ref, (err, ref)


@pytest.mark.parametrize("M,N,K", [(512, 768, 1024), (296, 520, 256), (1024, 256, 4096), (2048, 3072, 1024)])
@pytest.mark.parametrize("ak,bk", [(0, 0), (0, 1), (1, 0), (1, 1)])
@pytest.mark.parametrize("out_f32", [0, 1])
def test_gemm4w_bf16_layouts(cuda, M, N, K, ak, bk, out_f32):
    torch.manual_seed(M + N + K)
    a = torch.randn(M, K, device=cuda).to(BF)
    b = torch.randn(N, K, device=cuda).to(BF)
    ref = a.float() @ b.float().t()
    A = a.t().contiguous() if ak else a
    B = b.t().contiguous() if bk else b
    c = torch.empty(M, N, device=cuda, dtype=torch.float32 if out_f32 else BF)
    call("dtf_gemm4w", ptr(A), ptr(B), ptr(c), M, N, K, A.stride(0), B.stride(0), N, ak, bk, out_f32, 0, None,
         stream())
    _close(c, ref, 1e-5 if out_f32 else 1e-2)


def _fp8_bytes(shape, dev, fmt, gen):
    """Random finite OCP fp8 bytes (e4m3 = 0, e5m2 = 1) and their f32 values."""
    v = torch.randn(shape, generator=gen) * (2.0 if fmt == 0 else 8.0)
    f = v.to(torch.float8_e4m3fn if fmt == 0 else torch.float8_e5m2)
    return f.view(torch.uint8).to(dev), f.float().to(dev)


@pytest.mark.parametrize("M,N,K", [(512, 768, 1024), (8192, 1024, 1024), (300, 520, 256)])
@pytest.mark.parametrize("fmt_a", [0, 1])
def test_gemm4w_fp8(cuda, M, N, K, fmt_a):
    g = torch.Generator().manual_seed(M + K + fmt_a)
    aq, af = _fp8_bytes((M, K), cuda, fmt_a, g)
    bq, bf = _fp8_bytes((N, K), cuda, 0, g)
    scales = torch.tensor([0.5, 0.25], device=cuda)
    c = torch.empty(M, N, device=cuda, dtype=torch.float32)
    call("dtf_gemm4w", ptr(aq), ptr(bq), ptr(c), M, N, K, K, K, N, 0, 0, 1, 1 + fmt_a, ptr(scales), stream())
    _close(c, 0.125 * (af @ bf.t()), 1e-4)  # (f32 summation order)
