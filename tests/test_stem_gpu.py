"""The dedicated space-to-depth stem kernel (csrc/kernels/stem.hip): 4x4/1 conv over the s2d image, 64 channels,
with the BatchNorm partial sums of its bf16 output — against an f32 PyTorch conv of the same bf16 operands."""
import pytest
import torch

from distributed_tensorflow_amd.ops import conv as OC
from distributed_tensorflow_amd.ops._util import IntOut, K, ptr, stream

pytestmark = pytest.mark.gpu
BF = torch.bfloat16


@pytest.fixture(scope="module")
def cuda():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


@pytest.mark.parametrize("N,H,W", [(3, 84, 96), (2, 224, 224)])
def test_stem_fwd_matches_f32_conv(cuda, N, H, W):
    """P = 42 leaves a partial 8-row unit; 224 x 224 is the ResNet-50 shape (Q = 112)."""
    g = torch.Generator().manual_seed(5)
    img = torch.randn(N, 3, H, W, generator=g).to(cuda)
    w7 = (torch.randn(64, 7, 7, 4, generator=g) * 0.05).to(cuda)
    x = OC.image_to_s2d_bf16(img)  # [N, H/2+3, W/2+3, 16]
    w16 = OC.stem_s2d_filter(w7.to(BF))  # [64, 4, 4, 16]
    Hs, Ws = x.shape[1], x.shape[2]
    P, Q = Hs - 3, Ws - 3
    y = torch.empty(N, P, Q, 64, dtype=BF, device=cuda)
    part = torch.full((1024 * 128,), float("nan"), device=cuda)
    rows = IntOut()
    rc = K().dtf_stem_fwd(ptr(x), ptr(w16), ptr(y), ptr(part), rows.addr, N, Hs, Ws, 16, 64, 4, 4, P, Q, stream())
    assert rc == 0, rc
    torch.cuda.synchronize()
    ref = torch.nn.functional.conv2d(x.float().permute(0, 3, 1, 2), w16.float().permute(0, 3, 1, 2))
    ref = ref.permute(0, 2, 3, 1)
    err = (y.float() - ref).abs().max().item()
    assert err <= 0.01 * ref.abs().max().item(), err
    T = rows.value
    assert 0 < T <= 1024
    pr = part[:T * 128].view(T, 128).sum(0)
    yf = y.float().reshape(-1, 64)
    scale = yf.abs().sum(0).max().item()
    assert (pr[:64] - yf.sum(0)).abs().max().item() <= 1e-4 * scale
    assert torch.allclose(pr[64:], (yf * yf).sum(0), rtol=1e-4)


@pytest.mark.parametrize("N,P,Q", [(4, 1, 16), (3, 3, 16), (2, 1, 32)])
def test_stem_fwd_short_outputs_stay_in_stats_rows(cuda, N, P, Q):
    """Short outputs: the kernel may write at most ceil(N*P*Q/64) partial rows (the conv stats contract of its
    callers); the rows behind that must stay untouched, and the rows it wrote still sum to the statistics."""
    g = torch.Generator().manual_seed(7)
    Hs, Ws = P + 3, Q + 3
    x = torch.randn(N, Hs, Ws, 16, generator=g).to(BF).to(cuda)
    w16 = (torch.randn(64, 4, 4, 16, generator=g) * 0.05).to(BF).to(cuda)
    y = torch.empty(N, P, Q, 64, dtype=BF, device=cuda)
    cap = (N * P * Q + 63) // 64
    part = torch.full(((cap + 64) * 128,), float("nan"), device=cuda)
    rows = IntOut()
    rc = K().dtf_stem_fwd(ptr(x), ptr(w16), ptr(y), ptr(part), rows.addr, N, Hs, Ws, 16, 64, 4, 4, P, Q, stream())
    assert rc == 0, rc
    torch.cuda.synchronize()
    T = rows.value
    assert 0 < T <= cap, (T, cap)
    assert torch.isnan(part[T * 128:]).all(), "stem kernel wrote past its partial-statistics rows"
    ref = torch.nn.functional.conv2d(x.float().permute(0, 3, 1, 2), w16.float().permute(0, 3, 1, 2))
    ref = ref.permute(0, 2, 3, 1)
    assert (y.float() - ref).abs().max().item() <= 0.01 * ref.abs().max().item()
    pr = part[:T * 128].view(T, 128).sum(0)
    yf = y.float().reshape(-1, 64)
    assert (pr[:64] - yf.sum(0)).abs().max().item() <= 1e-4 * yf.abs().sum(0).max().item()


def test_stem_fwd_rejects_other_shapes(cuda):
    x = torch.zeros(1, 53, 53, 16, dtype=BF, device=cuda)  # Q = 50: not a multiple of 16
    w = torch.zeros(64, 4, 4, 16, dtype=BF, device=cuda)
    y = torch.empty(1, 50, 50, 64, dtype=BF, device=cuda)
    part = torch.empty(128 * 64, device=cuda)
    assert K().dtf_stem_fwd(ptr(x), ptr(w), ptr(y), ptr(part), None, 1, 53, 53, 16, 64, 4, 4, 50, 50, stream()) == -1
