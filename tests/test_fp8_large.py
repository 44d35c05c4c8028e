"""FP8 (OCP e4m3) GEMM on the 256x256 glds pipeline (large, chip-filling shapes) and the device-side exact
per-tensor weight scale, against dequantized f32 references."""
import pytest
import torch

from distributed_tensorflow_amd.ops import fp8
from distributed_tensorflow_amd.ops._util import call, ptr, stream, workspace

BF = torch.bfloat16


def close(a, b, tol):
    a, b = a.float(), b.float()
    err = (a - b).abs().max().item()
    ref = b.abs().max().item() + 1e-6
    assert err <= tol * ref, f"max err {err} vs ref scale {ref} (tol {tol})"


@pytest.mark.gpu
@pytest.mark.parametrize("M,N,K", [(4096, 4096, 1024), (8192, 3072, 1024), (2000, 1024, 4096)])
def test_fp8_gemm_large(cuda, M, N, K):
    torch.manual_seed(0)
    x = (torch.rand(M, K, device=cuda) * 2 - 1).to(BF)
    w = ((torch.rand(N, K, device=cuda) * 2 - 1) * 0.05).to(BF)
    ws = workspace(cuda)
    sw = torch.zeros(1, device=cuda)
    wq = torch.empty(N, K, dtype=torch.uint8, device=cuda)
    call("dtf_quant_fp8_exact", ptr(w), ptr(wq), w.numel(), ptr(sw), ptr(ws), stream())
    assert abs(sw.item() - w.float().abs().max().item() / 448.0) <= 1e-6 * max(1.0, sw.item())
    sx = (x.float().abs().max() / 448).reshape(1)
    xq = fp8.quantize(x, sx)
    scales = torch.cat([sx, sw])
    y = torch.empty(M, N, dtype=BF, device=cuda)
    call("dtf_gemm_fp8", ptr(xq), ptr(wq), ptr(y), None, None, ptr(scales), M, N, K, K, K, N, 0, -1, stream())
    ref = (xq.view(torch.float8_e4m3fn).float() * sx) @ (wq.view(torch.float8_e4m3fn).float() * sw).t()
    close(y, ref, 1e-2)
