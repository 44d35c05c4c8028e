"""Weight gradient of the space-to-depth ResNet stem on the persistent kernel (csrc/kernels/stemwgrad.hip,
ops.conv.stem_wgrad_raw): dW[k][a][b][c] = sum over output pixels of dY[n][h][w][k] * S[n][h + a][w + b][c] for the
valid 4x4/1 conv of the [N, Hs, Ws, 16] s2d image, the filter gradient resident in the accumulators, one dY row
image and a 16-slot ring of s2d rows in LDS, one f32 partial per block summed in a fixed order.

Checked against a plain PyTorch fp32 reference and against the general wgrad tiles (same sums, another f32
summation order), on shapes that put block boundaries inside and across images (the ring's restart path), the
widest row the kernel takes (Ws = 128), and for run-to-run determinism. The reference's op is the Conv2D weight
gradient of the ResNet-50 trainer's first layer (trainer/task.py:62-71)."""
import pytest
import torch

from distributed_tensorflow_amd.ops import conv as C
from distributed_tensorflow_amd.ops._util import K as kernels, ptr, stream, workspace

pytestmark = pytest.mark.gpu

BF = torch.bfloat16


def _ref(x, dy):
    N, Hs, Ws, _ = x.shape
    P, Q = Hs - 3, Ws - 3
    xf, df = x.float(), dy.float()
    out = torch.empty(64, 4, 4, 16, device=x.device)
    for a in range(4):
        for b in range(4):
            out[:, a, b, :] = torch.einsum("nhwk,nhwc->kc", df, xf[:, a:a + P, b:b + Q, :])
    return out


def _geom(N, Hs, Ws):
    return (N, Hs, Ws, 16, 64, 4, 4, Hs - 3, Ws - 3, 1, 1, 0, 0, 1, 1)


def _inputs(cuda, N, Hs, Ws, seed):
    g = torch.Generator(device="cpu").manual_seed(seed)
    x = torch.randn(N, Hs, Ws, 16, generator=g).to(BF).to(cuda)
    dy = torch.randn(N, Hs - 3, Ws - 3, 64, generator=g).to(BF).to(cuda)
    return x, dy


# (N, Hs, Ws): ResNet-50's 115 x 115 s2d image; fewer rows than blocks (one row per block, every block restarts
# its ring); several rows per block crossing image boundaries; the widest row (128 pixels: no zero pixels past Q)
@pytest.mark.parametrize("N,Hs,Ws", [(4, 115, 115), (3, 40, 33), (5, 70, 9), (64, 20, 20), (2, 31, 128),
                                     (16, 115, 115)])
def test_stem_wgrad_matches_reference(cuda, N, Hs, Ws):
    x, dy = _inputs(cuda, N, Hs, Ws, N * 1000 + Hs + Ws)
    dw = torch.full((64, 4, 4, 16), float("nan"), device=cuda)
    ws = workspace(cuda)
    rc = kernels().dtf_stem_wgrad(ptr(x), ptr(dy), ptr(dw), N, Hs, Ws, 0, ptr(ws), ws.numel(), stream())
    assert rc == 0
    ref = _ref(x, dy)
    torch.cuda.synchronize()
    scale = ref.abs().max().item()
    err = (dw - ref).abs().max().item()
    assert err <= 2e-5 * scale + 1e-3, (err, scale)
    gen = C.conv_wgrad_raw(x, dy, _geom(N, Hs, Ws))  # the general tiles
    assert (dw - gen).abs().max().item() <= 2e-5 * scale + 1e-3


def test_stem_wgrad_accumulates_and_is_deterministic(cuda):
    N, Hs, Ws = 8, 115, 115
    x, dy = _inputs(cuda, N, Hs, Ws, 7)
    base = torch.randn(64, 4, 4, 16, device=cuda)
    ws = workspace(cuda)
    outs = []
    for _ in range(2):
        dw = base.clone()
        assert kernels().dtf_stem_wgrad(ptr(x), ptr(dy), ptr(dw), N, Hs, Ws, 1, ptr(ws), ws.numel(), stream()) == 0
        outs.append(dw)
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1])
    ref = _ref(x, dy) + base
    assert (outs[0] - ref).abs().max().item() <= 2e-5 * ref.abs().max().item() + 1e-3


def test_stem_wgrad_raw_routes_and_falls_back(cuda):
    # the op picks the stem kernel for the s2d stem geometry and the general tiles for anything else (here Ws > 128)
    x, dy = _inputs(cuda, 1, 20, 140, 3)
    dw = C.stem_wgrad_raw(x, dy, _geom(1, 20, 140))
    ws = workspace(cuda)
    assert kernels().dtf_stem_wgrad(ptr(x), ptr(dy), ptr(dw), 1, 20, 140, 0, ptr(ws), ws.numel(), stream()) == -1
    ref = _ref(x, dy)
    assert (dw - ref).abs().max().item() <= 2e-5 * ref.abs().max().item() + 1e-3
    x, dy = _inputs(cuda, 2, 115, 115, 4)
    dw = C.stem_wgrad_raw(x, dy, _geom(2, 115, 115))
    ref = _ref(x, dy)
    assert (dw - ref).abs().max().item() <= 2e-5 * ref.abs().max().item() + 1e-3


@pytest.mark.parametrize("B,H", [(3, 224), (5, 60)])
def test_stem_wgrad_fused_is_bitwise_the_unfused_path(cuda, B, H, monkeypatch):
    """The stem's BN + ReLU + MaxPool backward applied inside the wgrad kernel (dtf_stem_wgrad_fused; the stem's dY
    is never stored) against the unfused path (maxpool_bn_bwd_apply writes dY, then the stem kernel): the dY values
    and the kernel's summation order are the same, so dW, dgamma and dbeta are bitwise equal."""
    from distributed_tensorflow_amd import ops
    g = torch.Generator().manual_seed(H + B)
    img = torch.randn(B, 3, H, H, generator=g).to(cuda)
    w = (torch.randn(64, 7, 7, 4, generator=g) * 0.05).to(cuda)
    gamma = (torch.rand(64, generator=g) + 0.5).to(cuda)
    beta = (torch.randn(64, generator=g) * 0.1).to(cuda)
    dyv = torch.randn(B, H // 4, H // 4, 64, generator=g).to(cuda)
    outs = []
    for fused in (False, True):
        monkeypatch.setattr(C, "_STEM_WGRAD_FUSED", fused)
        wd, gd, bd = (t.clone().requires_grad_(True) for t in (w, gamma, beta))
        rm, rv = torch.zeros(64, device=cuda), torch.ones(64, device=cuda)
        y = ops.conv_bn_maxpool(ops.image_to_s2d_bf16(img), wd, gd, bd, rm, rv, stride=(2, 2), pad=(3, 3), s2d=True)
        outs.append(torch.autograd.grad((y.float() * dyv).sum(), [wd, gd, bd]))
    torch.cuda.synchronize()
    for a, b in zip(*outs):
        assert torch.equal(a, b)
    assert outs[1][0].abs().max().item() > 0
