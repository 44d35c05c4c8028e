"""Two-pass ConvBN forward of the channel-expanding 1x1 conv (csrc/kernels/pwconv.hip MODE 1 + finalize + MODE 2,
dtf_conv_bn_apply_fwd): statistics pass, then the recomputed product with BatchNorm, residual (plain or itself a
deferred BatchNorm affine), ReLU and the 1-bit ReLU mask in the epilogue.

It must equal, BITWISE, the one-pass path it replaces (conv + statistics -> finalize -> dtf_bn_apply): the same bf16
conv output, statistics, running statistics, block output and mask. Both are also checked against a plain PyTorch
fp32 reference of conv -> training BatchNorm -> + residual -> ReLU."""
import pytest
import torch

from distributed_tensorflow_amd.ops._util import call, ptr, stream

pytestmark = pytest.mark.gpu

BF = torch.bfloat16
F32 = torch.float32


def _inputs(cuda, M, C, K, seed):
    g = torch.Generator(device="cpu").manual_seed(seed)
    x = torch.relu(torch.randn(M, C, generator=g)).to(BF).to(cuda)
    w = (torch.randn(K, C, generator=g) * C ** -0.5).to(BF).to(cuda)
    gamma = (torch.rand(K, generator=g) + 0.5).to(cuda)
    beta = (torch.randn(K, generator=g) * 0.1).to(cuda)
    res = torch.randn(M, K, generator=g).to(BF).to(cuda)
    rsc = (torch.rand(K, generator=g) + 0.5).to(cuda)
    rsh = (torch.randn(K, generator=g) * 0.1).to(cuda)
    return x, w, gamma, beta, res, rsc, rsh


def _one_pass(cuda, x, w, gamma, beta, res, raff, relu, M, C, K):
    yc = torch.empty(M, K, dtype=BF, device=cuda)
    part = torch.empty(((M + 63) // 64) * 2 * K, dtype=F32, device=cuda)
    rm, rv = torch.zeros(K, device=cuda), torch.ones(K, device=cuda)
    work = torch.empty(4 * K, device=cuda)
    sc, sh, mu, ist = work[:K], work[K:2 * K], work[2 * K:3 * K], work[3 * K:]
    call("dtf_conv_fwd_bn", ptr(x), ptr(w), ptr(yc), ptr(part), 1, M, 1, C, K, 1, 1, M, 1, 1, 1, 0, 0, 1, 1, -1,
         ptr(gamma), ptr(beta), ptr(rm), ptr(rv), 0.9, 1e-5, ptr(sc), ptr(sh), ptr(mu), ptr(ist), None, stream())
    out = torch.empty_like(yc)
    mb = torch.zeros(M * K // 8, dtype=torch.uint8, device=cuda)
    call("dtf_bn_apply", ptr(yc), ptr(sc), ptr(sh), ptr(res), ptr(out), M, K, int(relu), ptr(mb) if relu else None,
         ptr(raff[0]) if raff else None, ptr(raff[1]) if raff else None, stream())
    return yc, out, mb, work, rm, rv


def _two_pass(cuda, x, w, gamma, beta, res, raff, relu, M, C, K, keep_yc=True):
    yc = torch.full((M, K), float("nan"), dtype=BF, device=cuda) if keep_yc else None
    out = torch.full((M, K), float("nan"), dtype=BF, device=cuda)
    mb = torch.zeros(M * K // 8, dtype=torch.uint8, device=cuda)
    part = torch.empty(((M + 63) // 64) * 2 * K, dtype=F32, device=cuda)
    rm, rv = torch.zeros(K, device=cuda), torch.ones(K, device=cuda)
    work = torch.empty(4 * K, device=cuda)
    call("dtf_conv_bn_apply_fwd", ptr(x), ptr(w), ptr(yc), ptr(out), ptr(mb) if relu else None, ptr(res),
         ptr(raff[0]) if raff else None, ptr(raff[1]) if raff else None, M, C, K, int(relu), ptr(part), ptr(gamma),
         ptr(beta), ptr(rm), ptr(rv), 0.9, 1e-5, ptr(work[:K]), ptr(work[K:2 * K]), ptr(work[2 * K:3 * K]),
         ptr(work[3 * K:]), stream())
    return yc, out, mb, work, rm, rv


@pytest.mark.parametrize("M,C,K,res_kind,relu", [
    (1000, 64, 256, "plain", True), (5000, 128, 512, "affine", True), (3001, 256, 1024, "plain", True),
    (12544, 256, 2048, "none", False), (200003, 64, 256, "plain", True), (50176, 256, 1024, "affine", True),
    (4099, 128, 256, "none", True)])
def test_two_pass_matches_one_pass_bitwise(cuda, M, C, K, res_kind, relu):
    x, w, gamma, beta, res, rsc, rsh = _inputs(cuda, M, C, K, M + C + K)
    r = res if res_kind != "none" else None
    raff = (rsc, rsh) if res_kind == "affine" else None
    a = _one_pass(cuda, x, w, gamma, beta, r, raff, relu, M, C, K)
    b = _two_pass(cuda, x, w, gamma, beta, r, raff, relu, M, C, K)
    torch.cuda.synchronize()
    names = ("yc", "out", "mask", "scale/shift/mean/invstd", "running mean", "running var")
    for nm, u, v in zip(names, a, b):
        if nm == "mask" and not relu:
            continue
        assert torch.equal(u.view(torch.uint8) if u.dtype == BF else u, v.view(torch.uint8) if v.dtype == BF else v), nm
    # and against fp32 torch: conv -> training BN (biased batch variance) -> + residual -> ReLU
    y = x.float() @ w.float().t()
    mu, var = y.mean(0), y.var(0, unbiased=False)
    ref = (y - mu) * torch.rsqrt(var + 1e-5) * gamma + beta
    if r is not None:
        ref = ref + (r.float() * rsc + rsh if raff else r.float())
    if relu:
        ref = torch.relu(ref)
    torch.testing.assert_close(b[1].float(), ref, rtol=3e-2, atol=3e-2)


def test_two_pass_without_conv_output(cuda):
    """The backward-free form (Y = nullptr): only the block output and its mask are written."""
    M, C, K = 20000, 64, 256
    x, w, gamma, beta, res, _, _ = _inputs(cuda, M, C, K, 7)
    a = _one_pass(cuda, x, w, gamma, beta, res, None, True, M, C, K)
    b = _two_pass(cuda, x, w, gamma, beta, res, None, True, M, C, K, keep_yc=False)
    torch.cuda.synchronize()
    assert torch.equal(a[1].view(torch.uint8), b[1].view(torch.uint8))
    assert torch.equal(a[2], b[2])


def test_resnet_blocks_two_pass_match_one_pass(cuda, monkeypatch):
    """A stage-1-shaped projection block + identity block (c3: 64 -> 256 channels, both two-pass eligible; the
    projection residual arrives as a deferred BatchNorm affine) train step with the two-pass c3 forward equals the
    one-pass form bitwise: every gradient (input included)."""
    from distributed_tensorflow_amd.keras import initializers
    from distributed_tensorflow_amd.models import resnet as R
    from distributed_tensorflow_amd.ops import conv as OC
    x = torch.randn(8, 16, 16, 64, generator=torch.Generator().manual_seed(5)).to(cuda).to(BF)
    runs = {}
    for two in (False, True):
        monkeypatch.setattr(OC, "_TWO_PASS_PW", two)
        initializers.set_seed(3)
        blocks = [R.Bottleneck(64, stride=1, project=True), R.Bottleneck(64)]
        xx = x.clone().requires_grad_(True)
        h = xx
        for b in blocks:
            h = b(h, training=True)
        loss = (h.float() * torch.linspace(-1, 1, h.shape[-1], device=h.device)).square().mean()
        params = [w for b in blocks for w in b.trainable_weights]
        grads = torch.autograd.grad(loss, [xx] + params)
        stats = [w.detach().clone() for b in blocks for w in b.weights if not w.trainable]
        runs[two] = [h.detach().clone()] + [g.clone() for g in grads] + stats
    for a, b in zip(runs[False], runs[True]):
        assert torch.equal(a, b)
