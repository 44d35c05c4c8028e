"""Data gradient of a channel-reducing 1x1 conv on the persistent pointwise kernel (csrc/kernels/pwconv.hip MODE 3,
routed by conv_dgrad_impl in gemm.hip): dX = dY W (+ the parked residual gradient, its deferred ReLU mask applied),
with the BatchNorm-backward partial rows of dX for the BN(+ReLU) whose output the conv consumed.

dX must equal, BITWISE, the general GEMM tile's result (same bf16 product rounding, same staged beta arithmetic);
the BN partials (a different reduction order) must agree on their sums to fp32 accumulation accuracy. Both paths are
also checked against a plain PyTorch fp32 reference. The reference's op is the gradient of the Conv2D the ResNet-50
trainer builds (trainer/task.py:62-71)."""
import pytest
import torch

from distributed_tensorflow_amd.ops._util import call, ptr, stream

pytestmark = pytest.mark.gpu

BF = torch.bfloat16
F32 = torch.float32


def _dgrad(cuda, dy, wck, M, Kc, N, acc=None, amask=None, bn=None, pw=True, sub2=None, hw=None):
    """dtf_conv_dgrad_x of a 1x1 stride-1 conv (as [M,1,1], or [M/(H*W), H, W] with the compact stride-2 shortcut
    gradient sub2) with the pointwise route on or off."""
    import ctypes
    call("dtf_set_pw_dgrad", int(pw))
    try:
        dx = acc.clone() if acc is not None else torch.empty(M, N, dtype=BF, device=cuda)
        ws = torch.empty(16, dtype=BF, device=cuda)
        part = torch.full((((M + 63) // 64 + 1) * 2 * N,), float("nan"), dtype=F32, device=cuda) if bn else None
        rows = ctypes.c_int(0)
        bnp = (ptr(bn[0]), ptr(bn[1]), ptr(bn[2])) if bn else (None, None, None)
        H, W = hw if hw else (1, 1)
        call("dtf_conv_dgrad_x", ptr(dy), ptr(wck), ptr(dx), M // (H * W), H, W, N, Kc, 1, 1, H, W, 1, 1, 0, 0, 1, 1,
             1.0 if acc is not None else 0.0, ptr(ws), 16, *bnp, ptr(part),
             ctypes.addressof(rows) if bn else None, ptr(amask) if acc is not None else None, ptr(sub2), None, None,
             stream())
        torch.cuda.synchronize()
        sums = part[: rows.value * 2 * N].view(rows.value, 2 * N).sum(0) if bn else None
        return dx, sums, rows.value
    finally:
        call("dtf_set_pw_dgrad", 1)


def _bits(b):
    """[M, N] bool -> 1 bit per element, little-endian within a byte (the framework's mask layout)."""
    M, N = b.shape
    w = (1 << torch.arange(8, device=b.device, dtype=torch.int32))
    return (b.view(M, N // 8, 8).to(torch.int32) * w).sum(-1).to(torch.uint8).view(-1)


@pytest.mark.parametrize("M,Kc,N", [(5000, 64, 256), (3001, 128, 512), (12544, 256, 1024), (4099, 64, 512),
                                    (200003, 64, 256), (50176, 256, 1024), (100352, 128, 512)])
@pytest.mark.parametrize("kind", ["plain", "acc", "bn", "acc_bn"])
def test_pw_dgrad_matches_gemm_tile(cuda, M, Kc, N, kind):
    g = torch.Generator(device="cpu").manual_seed(M + Kc + N)
    dy = torch.randn(M, Kc, generator=g).to(BF).to(cuda)
    wck = (torch.randn(N, Kc, generator=g) * Kc ** -0.5).to(BF).to(cuda)
    acc = amask = bn = None
    if "acc" in kind:
        acc = torch.randn(M, N, generator=g).to(BF).to(cuda)
        keep = torch.rand(M, N, generator=g) > 0.4
        amask = _bits(keep.to(cuda))
    if "bn" in kind:
        x = torch.randn(M, N, generator=g).to(BF).to(cuda)
        on = torch.rand(M, N, generator=g) > 0.5
        mean = (torch.randn(N, generator=g) * 0.1).to(cuda)
        bn = (x, _bits(on.to(cuda)), mean)
    a, sa, ra = _dgrad(cuda, dy, wck, M, Kc, N, acc, amask, bn, pw=False)
    b, sb, rb = _dgrad(cuda, dy, wck, M, Kc, N, acc, amask, bn, pw=True)
    assert torch.equal(a.view(torch.int16), b.view(torch.int16)), "dX differs from the general tile"
    # fp32 reference of the stored values
    ref = dy.float() @ wck.float().t()
    if acc is not None:
        ref = ref + acc.float() * keep.to(cuda)
    assert torch.allclose(b.float(), ref, atol=3e-2, rtol=2e-2)
    if bn is not None:
        assert 0 < rb <= 256
        assert torch.isfinite(sb).all()
        scale = sa.abs().max().item() + 1.0
        assert torch.allclose(sa, sb, atol=1e-4 * scale, rtol=1e-4), (sa - sb).abs().max()
        dz = b.float() * on.to(cuda)
        rs = torch.cat([dz.sum(0), (dz * (bn[0].float() - mean)).sum(0)])
        assert torch.allclose(sb, rs, atol=1e-3 * scale, rtol=1e-3)


def test_pw_dgrad_route_taken(cuda):
    """The pointwise route writes one partial row per row slot (<= 256 rows), the general tile one per 128-row tile:
    the row count tells which ran."""
    M, Kc, N = 65536, 64, 256
    dy = torch.randn(M, Kc, device=cuda).to(BF)
    wck = torch.randn(N, Kc, device=cuda).to(BF)
    bn = (torch.randn(M, N, device=cuda).to(BF), torch.full((M * N // 8,), 255, dtype=torch.uint8, device=cuda),
          torch.zeros(N, device=cuda))
    _, _, r_gemm = _dgrad(cuda, dy, wck, M, Kc, N, bn=bn, pw=False)
    _, _, r_pw = _dgrad(cuda, dy, wck, M, Kc, N, bn=bn, pw=True)
    assert r_pw <= 256 < r_gemm


def test_pw_dgrad_block_gradients(cuda):
    """Three ResNet-50 stage-1 bottlenecks (width 64: every identity block's c1 dgrad, 64 -> 256 channels, takes the
    pointwise route with the parked residual gradient and the BN-backward partials of the previous block's output):
    the gradients with the route on and off agree to the f32 summation order of those partials."""
    from distributed_tensorflow_amd.keras import initializers
    from distributed_tensorflow_amd.models import resnet as R
    g = torch.Generator().manual_seed(11)
    x = torch.randn(16, 16, 16, 64, generator=g).to(cuda).to(BF)
    runs = {}
    for pw in (0, 1):
        call("dtf_set_pw_dgrad", pw)
        try:
            initializers.set_seed(3)
            blocks = [R.Bottleneck(64, stride=1, project=True), R.Bottleneck(64), R.Bottleneck(64)]
            xx = x.clone().requires_grad_(True)
            h = xx
            for b in blocks:
                h = b(h, training=True)
            loss = (h.float() * torch.linspace(-1, 1, h.shape[-1], device=cuda)).square().mean()
            params = [w for b in blocks for w in b.trainable_weights]
            runs[pw] = [t.float() for t in torch.autograd.grad(loss, [xx] + params)]
        finally:
            call("dtf_set_pw_dgrad", 1)
    worst = 0.0
    for a, b in zip(runs[0], runs[1]):
        assert torch.isfinite(b).all()
        worst = max(worst, (a - b).norm().item() / (a.norm().item() + 1e-12))
    assert worst < 1e-2, worst


@pytest.mark.parametrize("imgs,H,W,Kc,N", [(8, 56, 56, 128, 256), (6, 28, 28, 256, 512), (3, 14, 14, 64, 256)])
@pytest.mark.parametrize("with_bn", [False, True])
def test_pw_dgrad_compact_shortcut(cuda, imgs, H, W, Kc, N, with_bn):
    """The first block of ResNet-50 stages 2-3: c1's data gradient plus the compact [imgs, H/2, W/2, N] gradient of the
    stride-2 projection shortcut at the even pixels (never materialised full-size): bitwise the general tile's."""
    M = imgs * H * W
    g = torch.Generator(device="cpu").manual_seed(M + Kc)
    dy = torch.randn(M, Kc, generator=g).to(BF).to(cuda)
    wck = (torch.randn(N, Kc, generator=g) * Kc ** -0.5).to(BF).to(cuda)
    sub2 = torch.randn(imgs, H // 2, W // 2, N, generator=g).to(BF).to(cuda)
    bn = None
    if with_bn:
        on = torch.rand(M, N, generator=g) > 0.5
        bn = (torch.randn(M, N, generator=g).to(BF).to(cuda), _bits(on.to(cuda)),
              (torch.randn(N, generator=g) * 0.1).to(cuda))
    a, sa, _ = _dgrad(cuda, dy, wck, M, Kc, N, bn=bn, pw=False, sub2=sub2, hw=(H, W))
    b, sb, rb = _dgrad(cuda, dy, wck, M, Kc, N, bn=bn, pw=True, sub2=sub2, hw=(H, W))
    assert torch.equal(a.view(torch.int16), b.view(torch.int16))
    full = torch.zeros(imgs, H, W, N, device=cuda)
    full[:, ::2, ::2] = sub2.float()
    ref = dy.float() @ wck.float().t() + full.view(M, N)
    assert torch.allclose(b.float(), ref, atol=3e-2, rtol=2e-2)
    if with_bn:
        assert 0 < rb <= 256
        scale = sa.abs().max().item() + 1.0
        assert torch.allclose(sa, sb, atol=1e-4 * scale, rtol=1e-4)
