"""The persistent pointwise-conv forward (csrc/kernels/pwconv.hip): Y = X W^T in bf16 plus the per-column BN
statistics of the stored values, against a plain PyTorch fp32 reference of the same op — for every input width
it instantiates (64, 128, 256 channels), 1/2/4/8 column tiles, M tails that are not a multiple of the row tile,
and through dtf_conv_fwd's routing (a stride-1 1x1 conv with statistics takes this kernel)."""
import pytest
import torch

from distributed_tensorflow_amd.ops._util import IntOut, call, ptr, stream

pytestmark = pytest.mark.gpu

BF = torch.bfloat16


def _run(cuda, M, C, K, via_conv):
    g = torch.Generator(device="cpu").manual_seed(M + C + K)
    x = (torch.rand(M, C, generator=g) * 2 - 1).to(BF).to(cuda)
    w = ((torch.rand(K, C, generator=g) * 2 - 1) * 0.1).to(BF).to(cuda)
    y = torch.full((M, K), float("nan"), dtype=BF, device=cuda)
    part = torch.full((((M + 63) // 64) * 2 * K,), float("nan"), dtype=torch.float32, device=cuda)
    rows = IntOut()
    if via_conv:
        call("dtf_conv_fwd", ptr(x), ptr(w), ptr(y), None, ptr(part), rows.addr, 1, M, 1, C, K, 1, 1, M, 1, 1, 1, 0,
             0, 1, 1, 0, 0, -1, stream())
    else:
        call("dtf_pwconv_fwd", ptr(x), ptr(w), ptr(y), ptr(part), rows.addr, M, C, K, stream())
    torch.cuda.synchronize()
    ref = x.float() @ w.float().t()
    assert torch.isfinite(y.float()).all()
    torch.testing.assert_close(y.float(), ref, rtol=1e-2, atol=1e-2)
    R = rows.value
    assert 0 < R <= (M + 63) // 64
    st = part[:R * 2 * K].view(R, 2 * K).double().sum(0)
    yd = y.double()
    torch.testing.assert_close(st[:K], yd.sum(0), rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(st[K:], (yd * yd).sum(0), rtol=1e-4, atol=1e-3)
    return R


@pytest.mark.parametrize("M,C,K", [(1000, 64, 256), (5000, 128, 512), (3001, 256, 1024), (12544, 256, 2048),
                                   (50176, 256, 1024), (200003, 64, 256)])
def test_pwconv_matches_fp32_reference(cuda, M, C, K):
    _run(cuda, M, C, K, via_conv=False)


def test_conv_fwd_routes_pointwise_to_pwconv(cuda):
    # the general kernel leaves one partial row per 128-row M-tile; the persistent kernel one per row slot (<= 256)
    R = _run(cuda, 40000, 64, 256, via_conv=True)
    assert R <= 3 * 256
