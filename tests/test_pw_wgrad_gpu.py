"""Weight gradient of a 1x1 stride-1 conv on the persistent kernel (csrc/kernels/pwwgrad.hip, routed by
dtf_conv_wgrad): dW[K][C] = sum_p dY[p][k] X[p][c] with the whole filter tile in one block's accumulators and one f32
partial per block summed in a fixed order.

Checked against a plain PyTorch fp32 reference and against the general split-K tiles (same sums, a different f32
summation order), with and without accumulation into an existing gradient, and for run-to-run determinism. The
reference's op is the Conv2D weight gradient of the ResNet-50 trainer (trainer/task.py:62-71)."""
import pytest
import torch

from distributed_tensorflow_amd.ops._util import call, launch_counts, ptr, stream

pytestmark = pytest.mark.gpu

BF = torch.bfloat16


def _wgrad(cuda, x, dy, P, C, K, pw, out=None):
    call("dtf_set_pw_wgrad", 2 if pw else 0)
    try:
        dw = out.clone() if out is not None else torch.full((K, C), float("nan"), device=cuda)
        ws = torch.empty(32 << 20, dtype=torch.float32, device=cuda)
        call("dtf_conv_wgrad", ptr(x), ptr(dy), ptr(dw), P, 1, 1, C, K, 1, 1, 1, 1, 1, 1, 0, 0, 1, 1,
             int(out is not None), 0, -1, ptr(ws), ws.numel(), stream())
        torch.cuda.synchronize()
        return dw
    finally:
        call("dtf_set_pw_wgrad", 1)


@pytest.mark.parametrize("P,C,K", [(5000, 256, 64), (200003, 64, 256), (100000, 64, 64), (65536, 256, 64),
                                   (20000, 128, 128), (9000, 256, 128),
                                   (12345, 128, 256), (50177, 512, 128), (30011, 128, 512)])
@pytest.mark.parametrize("acc", [False, True])
def test_pw_wgrad_matches_reference(cuda, P, C, K, acc):
    g = torch.Generator(device="cpu").manual_seed(P + C + K)
    x = torch.randn(P, C, generator=g).to(BF).to(cuda)
    dy = torch.randn(P, K, generator=g).to(BF).to(cuda)
    out = torch.randn(K, C, generator=g).to(cuda) if acc else None
    new = _wgrad(cuda, x, dy, P, C, K, True, out)
    old = _wgrad(cuda, x, dy, P, C, K, False, out)
    ref = dy.float().t() @ x.float() + (out if acc else 0)
    scale = ref.abs().max().item()
    assert torch.isfinite(new).all()
    assert (new - ref).abs().max().item() <= 1e-4 * scale + 1e-3, (new - ref).abs().max().item()
    assert (new - old).abs().max().item() <= 1e-4 * scale + 1e-3
    again = _wgrad(cuda, x, dy, P, C, K, True, out)
    assert torch.equal(new, again)  # fixed-order reduction: deterministic


def test_pw_wgrad_route_skips_general_tiles(cuda):
    """The persistent route launches no general split-K tile (the launch counters stay put)."""
    P, C, K = 65536, 256, 64
    x = torch.randn(P, C, device=cuda).to(BF)
    dy = torch.randn(P, K, device=cuda).to(BF)
    before = launch_counts()
    _wgrad(cuda, x, dy, P, C, K, True)
    after = launch_counts()
    assert after["splitk"] == before["splitk"] and after["gemm_tile"] == before["gemm_tile"], (before, after)
