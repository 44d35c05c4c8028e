"""Lazy BatchNorm outputs (ops.conv_bn(lazy=True), gemm_core.h XF loaders): a bottleneck's first two ConvBNs never
write their BN+ReLU output; the consuming conv applies scale/shift + ReLU to the staged conv output in its forward
and weight-gradient operand loaders, and the backward recomputes the ReLU mask from the conv output.

The on-the-fly transform uses the same f32 formula and bf16 rounding as the bn_apply pass, so the kernels see the
same operand bits: conv outputs and weight gradients are compared bitwise (same kernel) or at bf16 rounding (the
materialised path may route a 3x3 conv to the 256-row kernel, a different f32 summation order)."""
import math

import pytest
import torch

from distributed_tensorflow_amd.models import resnet as R
from distributed_tensorflow_amd.ops import conv as OC
from distributed_tensorflow_amd.ops._util import call, ptr, stream, workspace

pytestmark = pytest.mark.gpu
BF = torch.bfloat16


def _coef(C, dev, seed):
    g = torch.Generator(device="cpu").manual_seed(seed)
    sc = (torch.rand(C, generator=g) + 0.5).to(dev)
    sh = (torch.randn(C, generator=g) * 0.5).to(dev)
    return sc, sh


# (N, H, W, Cin, K, R, S, stride, pad): 1x1 (K-contiguous LDS-DMA) and 3x3 (tap-uniform im2col, stride 1 and 2)
CASES = [(4, 14, 14, 64, 256, 1, 1, 1, 0), (2, 28, 28, 128, 128, 3, 3, 1, 1), (2, 28, 28, 64, 64, 3, 3, 2, 1),
         (3, 7, 9, 256, 64, 3, 3, 1, 1), (2, 30, 30, 64, 96, 1, 1, 1, 0)]


@pytest.mark.parametrize("case", CASES)
def test_conv_fwd_with_input_bn_matches_materialised(cuda, case):
    N, H, W, Cin, K, Rr, S, st, pd = case
    torch.manual_seed(3)
    z = torch.randn(N, H, W, Cin, device=cuda).to(BF)
    w = (torch.randn(K, Rr, S, Cin, device=cuda) / math.sqrt(Rr * S * Cin)).to(BF)
    sc, sh = _coef(Cin, cuda, 4)
    y = OC.materialize_bn(z, (sc, sh))
    ref = y.float()
    assert (ref - torch.relu(z.float() * sc + sh)).abs().max().item() <= 1e-2 * ref.abs().max().item()
    g = OC._geom(z, w, (st, st), (pd, pd), (1, 1))
    outs = []
    for xin, xf in ((y, None), (z, (sc, sh))):
        gm, bt = torch.rand(K, device=cuda) + 0.5, torch.randn(K, device=cuda)
        rm, rv = torch.zeros(K, device=cuda), torch.ones(K, device=cuda)
        scale, shift, mean, inv = (torch.empty(K, device=cuda) for _ in range(4))
        o = OC.conv_fwd_bn_raw(xin, w, g, gm, bt, rm, rv, 0.9, 1e-5, scale, shift, mean, inv, xf=xf)
        outs.append((o.float(), mean, inv))
    (o0, m0, i0), (o1, m1, i1) = outs
    err = (o0 - o1).abs().max().item()
    assert err <= 1e-2 * o0.abs().max().item(), err
    assert (m0 - m1).abs().max().item() <= 1e-3 * (m0.abs().max().item() + 1e-3)
    # and against the f32 conv of the BN+ReLU output
    f = OC._ref_conv(ref, w.float(), None, (st, st), (pd, pd), (1, 1))
    assert (o1 - f).abs().max().item() <= 2e-2 * f.abs().max().item()


WCASES = [(4, 14, 14, 64, 256, 1, 1, 1, 0), (2, 28, 28, 128, 128, 3, 3, 1, 1), (2, 28, 28, 64, 64, 3, 3, 2, 1),
          (2, 14, 14, 256, 64, 3, 3, 1, 1)]


@pytest.mark.parametrize("case", WCASES)
def test_conv_wgrad_with_input_bn_matches_materialised(cuda, case):
    N, H, W, Cin, K, Rr, S, st, pd = case
    torch.manual_seed(5)
    z = torch.randn(N, H, W, Cin, device=cuda).to(BF)
    w = torch.randn(K, Rr, S, Cin, device=cuda)
    g = OC._geom(z, w, (st, st), (pd, pd), (1, 1))
    dy = torch.randn(N, g[7], g[8], K, device=cuda).to(BF)
    sc, sh = _coef(Cin, cuda, 6)
    y = OC.materialize_bn(z, (sc, sh))
    d0 = OC.conv_wgrad_raw(y, dy, g)
    d1 = OC.conv_wgrad_raw(z, dy, g, xf=(sc, sh))
    assert torch.equal(d0, d1) or (d0 - d1).abs().max().item() <= 1e-3 * d0.abs().max().item()
    ref = torch.nn.grad.conv2d_weight(y.float().permute(0, 3, 1, 2), (K, Cin, Rr, S), dy.float().permute(0, 3, 1, 2),
                                      stride=st, padding=pd).permute(0, 2, 3, 1)
    assert (d1 - ref).abs().max().item() <= 1e-2 * ref.abs().max().item()


def test_dgrad_bn_stats_mask_from_coefficients(cuda):
    """The BN-backward statistics of a dgrad epilogue with the ReLU mask recomputed from the BN input (bnsc/bnsh)
    equal the ones taken with the bit mask that bn_apply would have written."""
    torch.manual_seed(7)
    N, H, W, C, K = 4, 14, 14, 64, 256
    dy = torch.randn(N, H, W, K, device=cuda).to(BF)
    w = torch.randn(K, 1, 1, C, device=cuda) / 16
    g = OC._geom(torch.empty(N, H, W, C), w, (1, 1), (0, 0), (1, 1))
    yc = torch.randn(N, H, W, C, device=cuda).to(BF)
    sc, sh = _coef(C, cuda, 8)
    mean = torch.randn(C, device=cuda) * 0.1
    y = torch.empty_like(yc)
    mbits = torch.empty(yc.numel() // 8, dtype=torch.uint8, device=cuda)
    call("dtf_bn_apply", ptr(yc), ptr(sc), ptr(sh), None, ptr(y), yc.numel() // C, C, 1, ptr(mbits), None, None,
         stream())
    res = []
    for mcoef in (None, (sc, sh)):
        src = OC._BNSource(yc, None if mcoef else mbits, mean, mcoef=mcoef)
        OC.conv_dgrad_raw(dy, w, g, bn=src)
        part, rows = src.part, src.rows
        res.append(part[:rows * 2 * C].view(rows, 2 * C).sum(0))
    assert torch.allclose(res[0], res[1], rtol=1e-5, atol=1e-4)


def _blocks():
    from distributed_tensorflow_amd.keras import initializers
    initializers.set_seed(3)
    return [R.Bottleneck(64, stride=2, project=True), R.Bottleneck(64)]


def _run(blocks, x):
    x = x.clone().requires_grad_(True)
    h = x
    for b in blocks:
        h = b(h, training=True)
    loss = (h.float() * torch.linspace(-1, 1, h.shape[-1], device=h.device)).square().mean()
    params = [w for b in blocks for w in b.trainable_weights]
    grads = torch.autograd.grad(loss, [x] + params)
    return [h.float()] + [gr.float() for gr in grads] + [b.c2.moving_mean.clone() for b in blocks]


def test_lazy_bottlenecks_match_materialised(cuda, monkeypatch):
    """Two bottleneck blocks (stride-2 projection + identity) with lazy c1/c2 outputs vs materialised ones: the
    forward output, every gradient and the running statistics agree (bitwise where the same kernels run), and the
    lazy run issues 4 fewer BN apply passes."""
    g = torch.Generator().manual_seed(11)
    x = torch.randn(4, 16, 16, 256, generator=g).to(cuda).to(BF)
    seen = []
    real = OC.call

    def spy(name, *args):
        seen.append(name)
        return real(name, *args)

    monkeypatch.setattr(OC, "call", spy)
    runs, applies = {}, {}
    for mode in ("0", "1", "1x1"):  # DTF_LAZY_BN: off / every bottleneck c1+c2 / only c2 (pointwise consumer)
        monkeypatch.setattr(OC, "_LAZY_BN", mode)
        seen.clear()
        runs[mode] = _run(_blocks(), x)
        torch.cuda.synchronize()
        applies[mode] = seen.count("dtf_bn_apply")
    assert applies["0"] - applies["1"] == 4, applies
    assert applies["0"] - applies["1x1"] == 2, applies
    for mode in ("1", "1x1"):
        worst = 0.0
        for a, b in zip(runs["0"], runs[mode]):
            s = a.abs().max().item() + 1e-6
            worst = max(worst, (a - b).abs().max().item() / s)
        assert worst < 2e-2, (mode, worst)
