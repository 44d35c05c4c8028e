"""BatchNorm finalize fused into the producing GEMM launch (gemm_core.h BnFin): the two-level last-arriver
reduction of the conv's partial rows plus the per-channel finalize, against the separate reduction + finalize
launches (forward) and against an f32 reference of the backward coefficients (dgrad)."""
import math

import pytest
import torch

from distributed_tensorflow_amd.ops import conv as C
from distributed_tensorflow_amd.ops._util import IntOut, call, crsk_shadow, ptr, stream, workspace

pytestmark = pytest.mark.gpu
BF = torch.bfloat16
F32 = torch.float32


@pytest.fixture(autouse=True)
def _fin_fused():
    """The in-launch finalize is opt-in (gemm.hip fin_on): switch it on for these tests only."""
    call("dtf_set_bn_fin_fused", 1)
    yield
    call("dtf_set_bn_fin_fused", 0)


def rnd(*shape, dev, scale=1.0):
    return (torch.randn(*shape, device=dev) * scale).to(BF)


def close(a, b, tol, what=""):
    a, b = a.float(), b.float()
    err = (a - b).abs().max().item()
    ref = b.abs().max().item() + 1e-6
    assert err <= tol * ref, f"{what}: max err {err} vs ref scale {ref} (tol {tol})"


# (N, H, W, Cin, K, R, S, stride, pad): 1x1 and 3x3 on the 128-row kernels, one wide long-K shape that routes to the
# 256-row conv256 kernel (N >= 256 columns, K >= 1024), partial M tiles, many tiles (two-level groups)
FWD_CASES = [(2, 16, 16, 64, 64, 3, 3, 1, 1), (3, 9, 9, 128, 256, 1, 1, 1, 0), (64, 28, 28, 256, 256, 3, 3, 1, 1),
             (2, 15, 15, 64, 128, 3, 3, 2, 1), (16, 28, 28, 64, 64, 1, 1, 1, 0), (1, 5, 7, 16, 32, 3, 3, 1, 1)]


@pytest.mark.parametrize("case", FWD_CASES)
def test_conv_fwd_fused_bn_finalize(cuda, case):
    N, H, W, Cin, K, R, S, st, pd = case
    torch.manual_seed(1)
    x = rnd(N, H, W, Cin, dev=cuda)
    w = (torch.randn(K, R, S, Cin, device=cuda) / math.sqrt(R * S * Cin)).to(BF)
    g = C._geom(x, w, (st, st), (pd, pd), (1, 1))
    P, Q = g[7], g[8]
    M = N * P * Q
    gamma = torch.rand(K, device=cuda) + 0.5
    beta = torch.randn(K, device=cuda)
    outs = []
    for fused_entry in (False, True):
        rm, rv = torch.full((K,), 0.3, device=cuda), torch.full((K,), 2.0, device=cuda)
        sc, sh, mu, inv = (torch.empty(K, device=cuda) for _ in range(4))
        y = torch.empty(N, P, Q, K, dtype=BF, device=cuda)
        part = torch.empty(((M + 63) // 64) * 2 * K, dtype=F32, device=cuda)
        if fused_entry:
            done = IntOut()
            call("dtf_conv_fwd_bn", ptr(x), ptr(w), ptr(y), ptr(part), N, H, W, Cin, K, R, S, P, Q, st, st, pd, pd,
                 1, 1, -1, ptr(gamma), ptr(beta), ptr(rm), ptr(rv), 0.9, 1e-5, ptr(sc), ptr(sh), ptr(mu), ptr(inv),
                 done.addr, None, None, stream())
            torch.cuda.synchronize()
            assert done.value == 1, "the conv launch did not finalize the BatchNorm"
        else:
            rows = IntOut()
            call("dtf_conv_fwd", ptr(x), ptr(w), ptr(y), None, ptr(part), rows.addr, N, H, W, Cin, K, R, S, P, Q,
                 st, st, pd, pd, 1, 1, 0, 0, -1, stream())
            call("dtf_bn_finalize", ptr(part), rows.value, ptr(gamma), ptr(beta), ptr(rm), ptr(rv), M, K, 0.9, 1e-5,
                 ptr(sc), ptr(sh), ptr(mu), ptr(inv), stream())
        outs.append((y.clone(), sc, sh, mu, inv, rm, rv))
    (y0, *a0), (y1, *a1) = outs
    assert torch.equal(y0, y1)
    for nm, u, v in zip(("scale", "shift", "mean", "invstd", "running_mean", "running_var"), a1, a0):
        close(u, v, 2e-5, nm)
    # and against the f32 statistics of the stored conv output
    yf = y1.float().reshape(M, K)
    close(a1[2], yf.mean(0), 1e-4, "mean vs f32")
    close(a1[3], torch.rsqrt(yf.var(0, unbiased=False) + 1e-5), 1e-3, "invstd vs f32")


DGRAD_CASES = [(2, 16, 16, 64, 64, 3, 3, 1, 1), (2, 12, 12, 256, 64, 1, 1, 1, 0), (64, 28, 28, 256, 1024, 1, 1, 1, 0),
               (4, 8, 8, 16, 32, 3, 3, 1, 1), (2, 16, 16, 64, 128, 3, 3, 2, 1)]


@pytest.mark.parametrize("case", DGRAD_CASES)
@pytest.mark.parametrize("accumulate", [0, 1])
def test_conv_dgrad_fused_bn_backward_finalize(cuda, case, accumulate):
    """dgrad + the BatchNorm backward finalize of its output's BatchNorm in one launch: dgamma/dbeta (+= with
    accumulate) and the apply coefficients, against f32 formulas over the stored dX. Strided dgrads run several
    launches and must report that they did not finalize."""
    N, H, W, Cin, K, R, S, st, pd = case
    torch.manual_seed(2)
    P, Q = (H + 2 * pd - R) // st + 1, (W + 2 * pd - S) // st + 1
    dy = rnd(N, P, Q, K, dev=cuda)
    w = torch.randn(K, R, S, Cin, device=cuda) / math.sqrt(R * S * Cin)
    M = N * H * W
    yc = rnd(N, H, W, Cin, dev=cuda)
    mask = torch.rand(M * Cin, device=cuda) > 0.4
    bits = (mask.view(-1, 8).to(torch.uint8) << torch.arange(8, device=cuda, dtype=torch.uint8)).sum(1).to(torch.uint8)
    mean = torch.randn(Cin, device=cuda) * 0.1
    invstd = torch.rand(Cin, device=cuda) + 0.5
    gamma = torch.rand(Cin, device=cuda) + 0.5
    dgamma0, dbeta0 = torch.randn(Cin, device=cuda), torch.randn(Cin, device=cuda)
    dgamma, dbeta = dgamma0.clone(), dbeta0.clone()
    coef = torch.zeros(3 * Cin, device=cuda)
    dx = torch.empty(N, H, W, Cin, dtype=BF, device=cuda)
    part = torch.empty(((M + 63) // 64 + st * st) * 2 * Cin, dtype=F32, device=cuda)
    rows, done = IntOut(), IntOut()
    ws = workspace(cuda)
    wc = crsk_shadow(w, K, R * S, Cin)
    call("dtf_conv_dgrad_bn", ptr(dy), ptr(wc), ptr(dx), N, H, W, Cin, K, R, S, P, Q, st, st, pd, pd, 1, 1, 0.0,
         ptr(ws), 2 * ws.numel(), ptr(yc), ptr(bits), ptr(mean), ptr(part), rows.addr, None, None, ptr(gamma),
         ptr(invstd), ptr(dgamma), ptr(dbeta), accumulate, ptr(coef), done.addr, None, None, stream())
    torch.cuda.synchronize()
    if st > 1:
        assert done.value == 0 and rows.value >= 1
        return
    assert done.value == 1
    dz = dx.float().reshape(M, Cin) * mask.view(M, Cin).float()
    sdz = dz.sum(0)
    sdx = (dz * (yc.float().reshape(M, Cin) - mean)).sum(0) * invstd
    base_g = dgamma0 if accumulate else torch.zeros_like(dgamma0)
    base_b = dbeta0 if accumulate else torch.zeros_like(dbeta0)
    close(dgamma - base_g, sdx, 1e-3, "dgamma")
    close(dbeta - base_b, sdz, 1e-3, "dbeta")
    k1, k2, k3 = gamma * invstd, sdz / M, sdx / M
    close(coef[:Cin], k1, 1e-5, "k1")
    close(coef[Cin:2 * Cin], -k1 * k3 * invstd, 2e-3, "kb")
    close(coef[2 * Cin:], k1 * (mean * invstd * k3 - k2), 2e-3, "kc")
