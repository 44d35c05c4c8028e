"""Numerics of every gfx950 HIP kernel against a plain PyTorch f32 reference of the same op."""
import math

import pytest
import torch

from distributed_tensorflow_amd import ops
from distributed_tensorflow_amd.ops import _util

pytestmark = pytest.mark.gpu

BF = torch.bfloat16
F32 = torch.float32


def rnd(*shape, dev, scale=1.0):
    return (torch.randn(*shape, device=dev) * scale).to(BF)


def close(a, b, tol):
    a = a.float()
    b = b.float()
    err = (a - b).abs().max().item()
    ref = b.abs().max().item() + 1e-6
    assert err <= tol * ref, f"max err {err} vs ref scale {ref} (tol {tol})"


@pytest.mark.parametrize("M,N,K", [(256, 256, 256), (1000, 520, 392), (64, 64, 64), (4096, 1024, 768),
                                   (130, 72, 1032), (8, 16, 40)])
@pytest.mark.parametrize("ak,bk", [(0, 0), (0, 1), (1, 1), (1, 0)])
def test_gemm_layouts(cuda, M, N, K, ak, bk):
    if ak and M % 8:
        pytest.skip()
    if bk and N % 8:
        pytest.skip()
    A = rnd(M, K, dev=cuda)
    B = rnd(N, K, dev=cuda)
    a_in = A.t().contiguous() if ak else A
    b_in = B.t().contiguous() if bk else B
    C = ops.gemm(a_in, b_in, a_kouter=bool(ak), b_kouter=bool(bk), out_dtype=torch.float32)
    ref = A.float() @ B.float().t()
    close(C, ref, 2e-3)


@pytest.mark.parametrize("M,N,K", [(2, 1000, 2048), (3, 10, 7), (13, 24, 5)])
def test_gemm_unaligned_padding(cuda, M, N, K):
    A, B = rnd(M, K, dev=cuda), rnd(N, K, dev=cuda)
    close(ops.gemm(A, B, out_dtype=torch.float32), A.float() @ B.float().t(), 2e-3)
    close(ops.gemm(A.t().contiguous(), B.t().contiguous(), a_kouter=True, b_kouter=True, out_dtype=torch.float32),
          A.float() @ B.float().t(), 2e-3)


def test_gemm_asymmetric_identity(cuda):
    # A = I with asymmetric B catches a transposed C write (guide §3)
    n = 128
    A = torch.eye(n, device=cuda).to(BF)
    B = torch.arange(n * n, device=cuda, dtype=torch.float32).reshape(n, n).remainder(251).to(BF)
    C = ops.gemm(A, B, out_dtype=torch.float32)
    assert torch.equal(C, B.float().t())


def test_gemm_epilogue_bias_act_stats(cuda):
    M, N, K = 512, 192, 256
    A, B = rnd(M, K, dev=cuda), rnd(N, K, dev=cuda)
    bias = torch.randn(N, device=cuda)
    stats = torch.zeros(2 * N, device=cuda)
    pre = torch.empty(M, N, dtype=BF, device=cuda)
    C = ops.gemm(A, B, bias=bias, act=2, aux=pre, stats=stats)
    z = A.float() @ B.float().t() + bias
    close(pre, z, 1e-2)
    close(C, torch.nn.functional.gelu(z, approximate="tanh"), 1e-2)
    y = C.float()
    close(stats[:N], y.sum(0), 1e-2)
    close(stats[N:], (y * y).sum(0), 1e-2)


def test_gemm_splitk_and_batched(cuda):
    A, B = rnd(64, 8192, dev=cuda), rnd(96, 8192, dev=cuda)
    C = ops.gemm(A, B, out_dtype=torch.float32, splitk=8)
    close(C, A.float() @ B.float().t(), 2e-3)
    a3, b3 = rnd(6, 100, 64, dev=cuda), rnd(6, 72, 64, dev=cuda)
    c3 = ops.gemm(a3, b3)
    close(c3, a3.float() @ b3.float().transpose(1, 2), 1e-2)


CONV_CASES = [
    # N, H, W, C, K, R, S, stride, pad
    (2, 56, 56, 64, 64, 1, 1, 1, 0),
    (2, 56, 56, 64, 64, 3, 3, 1, 1),
    (2, 56, 56, 128, 128, 3, 3, 2, 1),
    (2, 56, 56, 256, 512, 1, 1, 2, 0),
    (2, 224, 224, 8, 64, 7, 7, 2, 3),
    (3, 7, 7, 512, 512, 3, 3, 1, 1),
    (1, 13, 11, 24, 40, 3, 5, 1, 2),
    (1, 15, 13, 16, 32, 3, 3, 2, 1),   # odd sizes, strided dgrad phases
    (2, 9, 9, 32, 64, 1, 1, 2, 0),     # strided 1x1: 3 of 4 phases have no taps
    (1, 10, 11, 16, 16, 3, 3, 3, 1),   # stride 3
    (1, 12, 12, 32, 64, 3, 3, 1, 1),   # tap-uniform dgrad gather only (Kout % 64 == 0, C % 64 != 0)
    (2, 12, 10, 64, 32, 3, 3, 1, 1),   # tap-uniform fwd gather only
    (1, 17, 17, 128, 64, 3, 3, 2, 0),  # tap-uniform, unpadded stride-2 (phases with partial tap sets)
]


@pytest.mark.parametrize("case", CONV_CASES)
def test_conv_fwd_dgrad_wgrad(cuda, case):
    N, H, W, C, K, R, S, st, pd = case
    x = rnd(N, H, W, C, dev=cuda)
    w = (torch.randn(K, R, S, C, device=cuda) / math.sqrt(R * S * C)).requires_grad_(True)
    xg = x.clone().requires_grad_(True)
    y = ops.conv2d(xg, w, stride=(st, st), pad=(pd, pd))
    # reference on the bf16-rounded operands
    xr = x.float().permute(0, 3, 1, 2).requires_grad_(True)
    wr = w.detach().to(BF).float().permute(0, 3, 1, 2).requires_grad_(True)
    yr = torch.nn.functional.conv2d(xr, wr, stride=st, padding=pd)
    close(y.permute(0, 3, 1, 2), yr, 1e-2)
    g = torch.randn_like(yr)
    yr.backward(g)
    y.backward(g.permute(0, 2, 3, 1).to(BF))
    if C != 8:
        close(xg.grad.permute(0, 3, 1, 2), xr.grad, 2e-2)
    close(w.grad.permute(0, 3, 1, 2), wr.grad, 2e-2)


def test_conv_bn_relu_residual(cuda):
    N, H, W, C, K = 4, 28, 28, 64, 128
    x = rnd(N, H, W, C, dev=cuda).requires_grad_(True)
    w = (torch.randn(K, 3, 3, C, device=cuda) / 24).requires_grad_(True)
    gamma = (torch.rand(K, device=cuda) + 0.5).requires_grad_(True)
    beta = (torch.randn(K, device=cuda) * 0.1).requires_grad_(True)
    res = rnd(N, H, W, K, dev=cuda).requires_grad_(True)
    rm, rv = torch.zeros(K, device=cuda), torch.ones(K, device=cuda)
    y = ops.conv_bn(x, w, gamma, beta, rm, rv, pad=(1, 1), relu=True, residual=res, momentum=0.9, eps=1e-5)
    # reference
    xr = x.detach().float().requires_grad_(True)
    wr = w.detach().to(BF).float().requires_grad_(True)
    gr, br = gamma.detach().clone().requires_grad_(True), beta.detach().clone().requires_grad_(True)
    rr = res.detach().float().requires_grad_(True)
    yc = torch.nn.functional.conv2d(xr.permute(0, 3, 1, 2), wr.permute(0, 3, 1, 2), padding=1)
    yc = yc.to(BF).float()  # the kernel normalizes the bf16-stored conv output
    mean = yc.mean((0, 2, 3), keepdim=True)
    var = yc.var((0, 2, 3), unbiased=False, keepdim=True)
    yn = (yc - mean) / torch.sqrt(var + 1e-5) * gr.view(1, -1, 1, 1) + br.view(1, -1, 1, 1)
    out = torch.relu(yn + rr.permute(0, 3, 1, 2)).permute(0, 2, 3, 1)
    close(y, out, 2e-2)
    close(rm, 0.1 * mean.flatten(), 2e-2)
    g = torch.randn_like(out)
    out.backward(g)
    y.backward(g.to(BF))
    close(x.grad, xr.grad, 5e-2)
    close(w.grad, wr.grad, 5e-2)
    close(gamma.grad, gr.grad, 3e-2)
    close(beta.grad, br.grad, 3e-2)
    # the residual gradient is g * relu'(out): compare away from the bf16 rounding band around the ReLU kink
    away = (out.detach().abs() > 2e-2).float()
    close(res.grad * away, rr.grad * away, 2e-2)


def test_batchnorm_standalone(cuda):
    x = rnd(8, 14, 14, 256, dev=cuda, scale=2.0).requires_grad_(True)
    g = (torch.rand(256, device=cuda) + 0.5).requires_grad_(True)
    b = torch.zeros(256, device=cuda, requires_grad=True)
    y = ops.batch_norm(x, g, b, torch.zeros(256, device=cuda), torch.ones(256, device=cuda), relu=True, eps=1e-3)
    xr = x.detach().float().requires_grad_(True)
    gr, br = g.detach().clone().requires_grad_(True), b.detach().clone().requires_grad_(True)
    yr = torch.relu(torch.nn.functional.batch_norm(xr.permute(0, 3, 1, 2), None, None, gr, br, True, 0.0, 1e-3))
    yr = yr.permute(0, 2, 3, 1)
    close(y, yr, 2e-2)
    dy = torch.randn_like(yr)
    yr.backward(dy)
    y.backward(dy.to(BF))
    close(x.grad, xr.grad, 3e-2)
    close(g.grad, gr.grad, 2e-2)


def test_pools(cuda):
    x = rnd(4, 112, 112, 64, dev=cuda).requires_grad_(True)
    y = ops.max_pool2d(x)
    xr = x.detach().float().permute(0, 3, 1, 2).requires_grad_(True)
    yr = torch.nn.functional.max_pool2d(xr, 3, 2, 1)
    close(y.permute(0, 3, 1, 2), yr, 1e-6)
    g = torch.randn_like(yr).to(BF).float()
    yr.backward(g)
    y.backward(g.permute(0, 2, 3, 1).to(BF))
    close(x.grad.permute(0, 3, 1, 2), xr.grad, 1e-2)
    z = rnd(4, 7, 7, 2048, dev=cuda).requires_grad_(True)
    p = ops.global_avg_pool(z)
    close(p, z.float().mean((1, 2)), 1e-2)
    p.float().sum().backward()
    close(z.grad, torch.full_like(z.float(), 1 / 49), 1e-2)


def test_softmax_ce(cuda):
    logits = torch.randn(64, 1000, device=cuda).requires_grad_(True)
    labels = torch.randint(0, 1000, (64,), device=cuda)
    l = ops.sparse_softmax_cross_entropy(logits, labels)
    lr = torch.nn.functional.cross_entropy(logits.detach().requires_grad_(True), labels, reduction="none")
    close(l, lr, 1e-4)
    l.mean().backward()
    lg = logits.detach().clone().requires_grad_(True)
    torch.nn.functional.cross_entropy(lg, labels).backward()
    close(logits.grad, lg.grad, 1e-4)


def test_softmax_ce_bf16_odd_vocab(cuda):
    """bf16 logits with an odd vocabulary (rows start at every element offset mod 8: vector body + scalar
    head/tail), label smoothing, an ignored row (label -1) and per-row loss weights, vs f32 PyTorch."""
    rows, V = 37, 1001
    logits = (torch.randn(rows, V, device=cuda) * 3).to(BF).requires_grad_(True)
    labels = torch.randint(0, V, (rows,), device=cuda)
    labels[5] = -1
    wts = torch.rand(rows, device=cuda)
    l = ops.sparse_softmax_cross_entropy(logits, labels, label_smoothing=0.1)
    lf = logits.detach().float().requires_grad_(True)
    lr = torch.nn.functional.cross_entropy(lf, labels.clamp(min=0), reduction="none", label_smoothing=0.1)
    lr = torch.where(labels >= 0, lr, torch.zeros_like(lr))
    close(l, lr, 1e-3)
    (l * wts).sum().backward()
    (lr * wts).sum().backward()
    close(logits.grad, lf.grad, 2e-2)
    assert logits.grad[5].float().abs().max().item() == 0


def test_layernorm(cuda):
    x = rnd(512, 768, dev=cuda).requires_grad_(True)
    g = (torch.rand(768, device=cuda) + 0.5).requires_grad_(True)
    b = torch.randn(768, device=cuda).requires_grad_(True)
    y = ops.layer_norm(x, g, b, 1e-12)
    xr = x.detach().float().requires_grad_(True)
    gr, br = g.detach().clone().requires_grad_(True), b.detach().clone().requires_grad_(True)
    yr = torch.nn.functional.layer_norm(xr, (768,), gr, br, 1e-12)
    close(y, yr, 1e-2)
    dy = torch.randn_like(yr)
    yr.backward(dy)
    y.backward(dy.to(BF))
    close(x.grad, xr.grad, 2e-2)
    close(g.grad, gr.grad, 1e-2)
    close(b.grad, br.grad, 1e-2)


@pytest.mark.parametrize("M,D", [(3001, 1024), (257, 1536), (64, 2048), (20000, 768), (5, 264)])
def test_layernorm_shapes(cuda, M, D):
    x = rnd(M, D, dev=cuda).requires_grad_(True)
    g = (torch.rand(D, device=cuda) + 0.5).requires_grad_(True)
    b = torch.randn(D, device=cuda).requires_grad_(True)
    y = ops.layer_norm(x, g, b, 1e-5)
    xr = x.detach().float().requires_grad_(True)
    gr, br = g.detach().clone().requires_grad_(True), b.detach().clone().requires_grad_(True)
    yr = torch.nn.functional.layer_norm(xr, (D,), gr, br, 1e-5)
    close(y, yr, 1e-2)
    dy = torch.randn_like(yr)
    yr.backward(dy)
    y.backward(dy.to(BF))
    close(x.grad, xr.grad, 2e-2)
    close(g.grad, gr.grad, 1e-2)
    close(b.grad, br.grad, 1e-2)


@pytest.mark.parametrize("M,N", [(16384, 768), (7, 3072), (1000, 776), (33, 30528)])
def test_colsum(cuda, M, N):
    x = rnd(M, N, dev=cuda).to(BF)
    out = ops.linalg.colsum(x)
    close(out, x.float().sum(0), 1e-3)
    out2 = torch.ones(N, device=cuda)
    ops.linalg.colsum(x, out=out2, accumulate=True)
    close(out2, x.float().sum(0) + 1, 1e-3)


def test_embedding_types_random_grad(cuda):
    V, S, B, D = 3000, 128, 8, 128
    table = torch.randn(V, D, device=cuda).requires_grad_(True)
    pos = torch.randn(256, D, device=cuda).requires_grad_(True)
    typ = torch.randn(2, D, device=cuda).requires_grad_(True)
    ids = torch.randint(0, 50, (B, S), device=cuda)  # heavy repetition
    tids = torch.randint(0, 2, (B, S), device=cuda)
    y = ops.embedding(ids, table, pos, tids, typ)
    dy = torch.randn(B, S, D, device=cuda).to(BF)
    y.backward(dy)
    t_r, p_r, y_r = (t.detach().to(BF).float().requires_grad_(True) for t in (table, pos, typ))
    yr = t_r[ids] + p_r[:S][None] + y_r[tids]
    close(y, yr, 1e-2)
    yr.backward(dy.float())
    close(table.grad, t_r.grad, 1e-3)
    close(pos.grad, p_r.grad, 1e-3)
    close(typ.grad, y_r.grad, 1e-3)


def test_softmax_masked(cuda):
    x = rnd(2, 4, 128, 128, dev=cuda).requires_grad_(True)
    y = ops.softmax(x, scale=0.125, causal=True)
    xr = x.detach().float().requires_grad_(True)
    yr = ops.nn.softmax(xr, scale=0.125, causal=True)  # CPU-path math on a cuda f32 tensor
    close(y, yr, 1e-2)


def test_dense_fwd_bwd(cuda):
    x = rnd(256, 768, dev=cuda).requires_grad_(True)
    w = (torch.randn(3072, 768, device=cuda) * 0.02).requires_grad_(True)
    b = torch.randn(3072, device=cuda).requires_grad_(True)
    from distributed_tensorflow_amd.ops._util import call_log
    with call_log() as calls:
        y = ops.dense(x, w, b, act="gelu")
    assert calls["dtf_gemm"] == 1, calls  # the forward product on our GEMM (no library route)
    xr = x.detach().float().requires_grad_(True)
    wr = w.detach().to(BF).float().requires_grad_(True)
    br = b.detach().clone().requires_grad_(True)
    yr = torch.nn.functional.gelu(xr @ wr.t() + br, approximate="tanh")
    close(y, yr, 2e-2)
    dy = torch.randn_like(yr)
    yr.backward(dy)
    with call_log() as calls:
        y.backward(dy.to(BF))
    assert calls["dtf_gemm"] == 2, calls  # data gradient and weight gradient on our GEMM
    close(x.grad, xr.grad, 3e-2)
    close(w.grad, wr.grad, 3e-2)
    close(b.grad, br.grad, 3e-2)


def test_embedding(cuda):
    table = torch.randn(1000, 64, device=cuda).requires_grad_(True)
    pos = torch.randn(32, 64, device=cuda).requires_grad_(True)
    ids = torch.randint(0, 1000, (4, 32), device=cuda)
    y = ops.embedding(ids, table, pos)
    yr = table.detach().to(BF).float()[ids] + pos.detach().to(BF).float()[None]
    close(y, yr, 1e-2)
    y.float().sum().backward()
    cnt = torch.bincount(ids.flatten(), minlength=1000).float()
    close(table.grad, cnt[:, None].expand(-1, 64), 1e-6)
    close(pos.grad, torch.full_like(pos, 4.0), 1e-6)


@pytest.mark.parametrize("kind", ["sgd", "adam", "adagrad", "adadelta", "ftrl", "rmsprop"])
def test_optimizers_match_reference(cuda, kind):
    from distributed_tensorflow_amd.keras import optimizers as O
    n = 10007
    p0 = torch.randn(n)
    gs = [torch.randn(n) for _ in range(5)]
    ref = O.reference_update(kind, p0.clone(), gs, lr=0.01)
    p = p0.clone().to(cuda)
    opt = O.get(kind, learning_rate=0.01)
    out = O.fused_update_for_test(opt, p, [g.to(cuda) for g in gs])
    close(out.cpu(), ref, 1e-4)


def test_fp8_quant_and_gemm(cuda):
    from distributed_tensorflow_amd.ops import fp8
    M, N, K = 512, 384, 1024
    x = rnd(M, K, dev=cuda)
    w = rnd(N, K, dev=cuda, scale=0.05)
    sx = (x.float().abs().max() / 448).reshape(1)
    sw = (w.float().abs().max() / 448).reshape(1)
    amax = torch.zeros(1, device=cuda)
    xq = fp8.quantize(x, sx, amax)
    wq = fp8.quantize(w, sw)
    assert abs(amax.item() - x.float().abs().max().item()) < 1e-6
    # decode with torch's OCP e4m3 type and compare to the quantized reference
    xd = xq.view(torch.float8_e4m3fn).float() * sx
    assert (xd - x.float()).abs().max().item() <= 0.07 * x.float().abs().max().item()
    scales = torch.cat([sx, sw])
    y = torch.empty(M, N, dtype=BF, device=cuda)
    from distributed_tensorflow_amd.ops._util import call, ptr, stream
    call("dtf_gemm_fp8", ptr(xq), ptr(wq), ptr(y), None, None, ptr(scales), M, N, K, K, K, N, 0, -1, stream())
    ref = (xq.view(torch.float8_e4m3fn).float() * sx) @ (wq.view(torch.float8_e4m3fn).float() * sw).t()
    close(y, ref, 1e-2)


def test_fp8_dense_layer_trains(cuda):
    from distributed_tensorflow_amd.models.transformer import _Proj
    torch.manual_seed(0)
    layer = _Proj(256, activation="gelu", fp8=True)
    x = rnd(128, 512, dev=cuda)
    y = layer(x)
    ref = torch.nn.functional.gelu(x.float() @ layer.kernel.detach().to(BF).float().t() + layer.bias.detach(),
                                   approximate="tanh")
    close(y, ref, 8e-2)
    y.float().sum().backward()
    assert layer.kernel.grad is not None and torch.isfinite(layer.kernel.grad).all()


def test_conv_bn_direct_arena_grads(cuda):
    """Inside direct_grads() ConvBN accumulates dW/dgamma/dbeta straight into the arena gradient views and
    fires the post-accumulate hooks; the result equals the regular autograd path (twice: accumulation)."""
    from distributed_tensorflow_amd.ops._util import direct_grads
    from distributed_tensorflow_amd.variables import ParamArena, Variable
    N, H, W, C, K = 2, 14, 14, 32, 64
    x = rnd(N, H, W, C, dev=cuda)
    results = []
    for direct in (False, True):
        torch.manual_seed(3)
        w = Variable((torch.randn(K, 3, 3, C) / 20).to(cuda), name="w")
        gm = Variable(torch.rand(K).to(cuda) + 0.5, name="g")
        bt = Variable(torch.zeros(K).to(cuda), name="b")
        arena = ParamArena([w, gm, bt], device=cuda)
        fired = []
        for v in (w, gm, bt):
            v.register_post_accumulate_grad_hook(lambda p: fired.append(p.name))
        rm, rv = torch.zeros(K, device=cuda), torch.ones(K, device=cuda)
        for _ in range(2):
            y = ops.conv_bn(x, w, gm, bt, rm, rv, pad=(1, 1), relu=True)
            loss = y.float().square().mean()
            if direct:
                with direct_grads():
                    loss.backward()
            else:
                loss.backward()
        assert sorted(fired) == sorted(["w", "g", "b"] * 2)
        results.append(arena.grad.clone())
    close(results[1], results[0], 1e-5)


@pytest.mark.parametrize("case", [(2, 16, 16, 64, 64, 3, 3, 1, 1), (2, 16, 16, 64, 128, 3, 3, 2, 1),
                                  (2, 12, 12, 256, 64, 1, 1, 1, 0), (4, 8, 8, 16, 32, 3, 3, 1, 1)])
@pytest.mark.parametrize("beta", [0.0, 1.0])
@pytest.mark.parametrize("tile", [-1, 11])
def test_conv_dgrad_fused_bn_backward_stats(cuda, case, beta, tile):
    """dtf_conv_dgrad's BN-backward epilogue: partial rows of sum(dz), sum(dz*(x-mean)) with dz = dX*mask."""
    from distributed_tensorflow_amd.ops import conv as C
    from distributed_tensorflow_amd.ops._util import IntOut, call, crsk_shadow, ptr, stream, workspace
    N, H, W, Cin, K, R, S, st, pd = case
    dy = rnd(N, (H + 2 * pd - R) // st + 1, (W + 2 * pd - S) // st + 1, K, dev=cuda)
    w = torch.randn(K, R, S, Cin, device=cuda) / math.sqrt(R * S * Cin)
    x = rnd(N, H, W, Cin, dev=cuda)
    g = C._geom(x, w, (st, st), (pd, pd), (1, 1))
    M = N * H * W
    yc = rnd(N, H, W, Cin, dev=cuda)
    mask = torch.rand(M * Cin, device=cuda) > 0.4
    bits = (mask.view(-1, 8).to(torch.uint8) << torch.arange(8, device=cuda, dtype=torch.uint8)).sum(1).to(torch.uint8)
    mean = torch.randn(Cin, device=cuda) * 0.1
    acc0 = rnd(N, H, W, Cin, dev=cuda)
    dx = acc0.clone()
    part = torch.empty(((M + 63) // 64 + st * st) * 2 * Cin, dtype=torch.float32, device=cuda)
    rows = IntOut()
    ws = workspace(cuda)
    wc = crsk_shadow(w, K, R * S, Cin)
    call("dtf_conv_dgrad", ptr(dy), ptr(wc), ptr(dx), N, H, W, Cin, K, R, S, g[7], g[8], st, st, pd, pd, 1, 1, 0,
         beta, tile, ptr(ws), 2 * ws.numel(), ptr(yc), ptr(bits), ptr(mean), ptr(part), rows.addr, None, stream())
    T = rows.value
    assert T >= 1
    p = part[:T * 2 * Cin].view(T, 2 * Cin).sum(0)
    dz = dx.float().reshape(M, Cin) * mask.view(M, Cin).float()
    s_ref = dz.sum(0)
    q_ref = (dz * (yc.float().reshape(M, Cin) - mean)).sum(0)
    close(p[:Cin], s_ref, 1e-3)
    close(p[Cin:], q_ref, 1e-3)


@pytest.mark.parametrize("tile", [0, 2, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16])
@pytest.mark.parametrize("case", [(2, 14, 14, 64, 128, 3, 3, 1, 1), (3, 9, 9, 128, 64, 1, 1, 1, 0),
                                  (2, 15, 15, 64, 64, 3, 3, 2, 1), (5, 13, 11, 128, 192, 3, 3, 1, 1)])
def test_conv_staging_pipelines_agree(cuda, case, tile):
    """Every staging pipeline (register-staged single/double LDS buffer, LDS-DMA single/double buffer, the
    256-row triple-buffered conv256 kernel: tiles 11-13) and tile shape computes bitwise the same conv forward
    and data gradient (same per-element K order)."""
    from distributed_tensorflow_amd.ops import conv as C
    from distributed_tensorflow_amd.ops._util import call, crsk_shadow, ptr, stream, workspace
    N, H, W, Cin, K, R, S, st, pd = case
    x = rnd(N, H, W, Cin, dev=cuda)
    w = torch.randn(K, R, S, Cin, device=cuda) / math.sqrt(R * S * Cin)
    g = C._geom(x, w, (st, st), (pd, pd), (1, 1))
    P, Q = g[7], g[8]
    w16 = w.to(BF)

    def fwd(t):
        y = torch.empty(N, P, Q, K, dtype=BF, device=cuda)
        call("dtf_conv_fwd", ptr(x), ptr(w16), ptr(y), None, None, None, N, H, W, Cin, K, R, S, P, Q, st, st, pd, pd,
             1, 1, 0, 0, t, stream())
        return y

    dy = rnd(N, P, Q, K, dev=cuda)
    wc = crsk_shadow(w, K, R * S, Cin)
    ws = workspace(cuda)

    def dgrad(t):
        dx = torch.empty_like(x)
        call("dtf_conv_dgrad", ptr(dy), ptr(wc), ptr(dx), N, H, W, Cin, K, R, S, P, Q, st, st, pd, pd, 1, 1, 0, 0.0, t,
             ptr(ws), 2 * ws.numel(), None, None, None, None, None, None, stream())
        return dx

    assert torch.equal(fwd(tile), fwd(-1))
    assert torch.equal(dgrad(tile), dgrad(-1))
    yr = torch.nn.functional.conv2d(x.float().permute(0, 3, 1, 2), w16.float().permute(0, 3, 1, 2), stride=st,
                                    padding=pd)
    close(fwd(tile).permute(0, 3, 1, 2), yr, 1e-2)


@pytest.mark.parametrize("tile", [7, 8, 9, 10])
@pytest.mark.parametrize("case", [(2, 14, 14, 64, 128, 3, 3, 1, 1), (3, 9, 9, 128, 64, 1, 1, 1, 0),
                                  (2, 15, 15, 64, 64, 3, 3, 2, 1), (2, 12, 12, 64, 256, 1, 1, 2, 0)])
def test_conv_wgrad_lds_dma_matches(cuda, case, tile, monkeypatch):
    """Weight gradient with LDS-DMA staged K-outer operands (DTF_GLDS_WGRAD path, forced tiles) equals the
    register-staged kernel bitwise (same K order) and the f32 reference."""
    from distributed_tensorflow_amd.ops import conv as C
    from distributed_tensorflow_amd.ops._util import call, ptr, stream, workspace
    N, H, W, Cin, K, R, S, st, pd = case
    x = rnd(N, H, W, Cin, dev=cuda)
    g = C._geom(x, torch.empty(K, R, S, Cin), (st, st), (pd, pd), (1, 1))
    P, Q = g[7], g[8]
    dy = rnd(N, P, Q, K, dev=cuda)
    ws = workspace(cuda)

    def wgrad(t):
        dw = torch.zeros(K, R, S, Cin, device=cuda)
        call("dtf_conv_wgrad", ptr(x), ptr(dy), ptr(dw), N, H, W, Cin, K, R, S, P, Q, st, st, pd, pd, 1, 1, 0, 1, t,
             ptr(ws), ws.numel(), stream())
        return dw
    got = wgrad(tile)
    base = wgrad(0)
    assert torch.equal(got, base)
    xr = x.float().permute(0, 3, 1, 2).requires_grad_(True)
    wr = torch.zeros(K, Cin, R, S, device=cuda, requires_grad=True)
    torch.nn.functional.conv2d(xr, wr, stride=st, padding=pd).backward(dy.float().permute(0, 3, 1, 2))
    close(got.permute(0, 3, 1, 2), wr.grad, 1e-2)


def test_add_dropout_matches_two_kernel_form(cuda):
    """x + dropout(f) in one pass == add(x, dropout(f)) with the same seed, bit for bit, forward and backward;
    the realised keep rate matches."""
    x = rnd(64, 768, dev=cuda).requires_grad_(True)
    f = rnd(64, 768, dev=cuda).requires_grad_(True)
    dy = rnd(64, 768, dev=cuda)
    y1 = ops.add_dropout(x, f, 0.1, training=True, seed=1234)
    gx1, gf1 = torch.autograd.grad(y1, [x, f], dy)
    y2 = ops.add(x, ops.dropout(f, 0.1, training=True, seed=1234))
    gx2, gf2 = torch.autograd.grad(y2, [x, f], dy)
    assert torch.equal(y1, y2) and torch.equal(gx1, gx2) and torch.equal(gf1, gf2)
    kept = (gf1 != 0).float().mean().item()
    assert abs(kept - 0.9) < 0.01


def test_bert_layer_residual_grad_link(cuda, monkeypatch):
    """BERT layer with the residual gradients joined inside the branch projections' data-gradient GEMMs
    (ResidualGradLink through ops.add_dropout / ops.dense) == autograd summing them: same gradients up to the one
    bf16 rounding of the sum."""
    from distributed_tensorflow_amd.keras import initializers
    from distributed_tensorflow_amd.models import transformer as T
    g = torch.Generator().manual_seed(3)
    x = torch.randn(2, 64, 128, generator=g).to(cuda).to(BF)
    dy = torch.randn(2, 64, 128, generator=g).to(cuda)
    from distributed_tensorflow_amd.ops._util import launch_counts, launch_delta
    res = {}
    for link in (False, True):
        before = launch_counts()
        monkeypatch.setattr(T, "RES_LINK", link)
        from distributed_tensorflow_amd.ops import mha as _mha, nn as _nn
        _nn._seed_counter[0], _mha._seed_counter[0] = 0x5EED, 0  # same dropout masks in both runs
        initializers.set_seed(7)
        layer = T.BertLayer(hidden=128, heads=2, ffn=256, dropout=0.1)
        xx = x.clone().requires_grad_(True)
        y = layer(xx, training=True)
        grads = torch.autograd.grad((y.float() * dy).sum(), [xx] + list(layer.trainable_weights))
        res[link] = [t.float().cpu() for t in grads]
        # with the link, the branch projections' data-gradient GEMMs add the parked residual gradient (bf16 beta = 1)
        beta = launch_delta(before)["beta_bf16"]
        assert (beta >= 2) if link else (beta == 0), (link, beta)
    for a, b in zip(res[False], res[True]):
        assert (a - b).abs().max().item() <= 2e-2 * a.abs().max().item() + 1e-6


@pytest.mark.parametrize("tile", [11, 12, 13, 14])
@pytest.mark.parametrize("case", [(2, 14, 14, 64, 128, 3, 3, 1, 1), (3, 9, 9, 128, 64, 1, 1, 1, 0),
                                  (2, 15, 15, 64, 64, 3, 3, 2, 1), (2, 12, 12, 64, 256, 1, 1, 2, 0),
                                  (4, 7, 9, 16, 64, 4, 4, 1, 0)])
def test_conv_wgrad_conv256_matches_reference(cuda, case, tile):
    """Weight gradient on the 256-row pipelined kernel (dW^T = X^T dY over split-K slabs, reduced and
    transposed; forced tiles 11-13) against the f32 reference, accumulating into an existing gradient."""
    from distributed_tensorflow_amd.ops import conv as C
    from distributed_tensorflow_amd.ops._util import call, ptr, stream, workspace
    N, H, W, Cin, K, R, S, st, pd = case
    x = rnd(N, H, W, Cin, dev=cuda)
    g = C._geom(x, torch.empty(K, R, S, Cin), (st, st), (pd, pd), (1, 1))
    P, Q = g[7], g[8]
    dy = rnd(N, P, Q, K, dev=cuda)
    ws = workspace(cuda)
    base = torch.randn(K, R, S, Cin, device=cuda)
    dw = base.clone()
    call("dtf_conv_wgrad", ptr(x), ptr(dy), ptr(dw), N, H, W, Cin, K, R, S, P, Q, st, st, pd, pd, 1, 1, 1, 0, tile,
         ptr(ws), ws.numel(), stream())
    xr = x.float().permute(0, 3, 1, 2).requires_grad_(True)
    wr = torch.zeros(K, Cin, R, S, device=cuda, requires_grad=True)
    torch.nn.functional.conv2d(xr, wr, stride=st, padding=pd).backward(dy.float().permute(0, 3, 1, 2))
    close((dw - base).permute(0, 3, 1, 2), wr.grad, 1e-2)


@pytest.mark.parametrize("case", [(64, 28, 128, 256, 1), (8, 28, 128, 256, 2), (4, 13, 256, 512, 1),
                                  (3, 14, 512, 512, 2)])
def test_conv_fwd_w4_im2col_bn_stats(cuda, case):
    """3x3 convolutions with >= 128 output channels take the 4-wave kernel with the implicit-GEMM loader
    (gemm_w4.hip W4Im2col: per-row tap masks, padding read as zeros by the buffer range check) and its BN-statistics
    epilogue: output against the f32 reference and the partial rows against the column sums / sums of squares, on
    strided, odd-sized (partial 256-row tiles) and 256- / 128-wide tile shapes; launch-counted."""
    from distributed_tensorflow_amd.ops import conv as C
    from distributed_tensorflow_amd.ops._util import launch_counts, launch_delta
    N, H, Cin, K, st = case
    x = rnd(N, H, H, Cin, dev=cuda)
    w = torch.randn(K, 3, 3, Cin, device=cuda) / math.sqrt(9 * Cin)
    g = C._geom(x, w, (st, st), (1, 1), (1, 1))
    before = launch_counts()
    y, part, rows = C.conv_fwd_raw(x, w.to(BF), g, stats=True)
    torch.cuda.synchronize()
    d = launch_delta(before)
    assert d["w4_256"] + d["w4_128"] == 1, d
    yr = torch.nn.functional.conv2d(x.float().permute(0, 3, 1, 2), w.to(BF).float().permute(0, 3, 1, 2), padding=1,
                                    stride=st)
    close(y.permute(0, 3, 1, 2).float(), yr, 1e-2)
    p = part[:rows * 2 * K].view(rows, 2 * K).sum(0)
    yf = y.float().reshape(-1, K)
    close(p[:K], yf.sum(0), 1e-3)
    close(p[K:], (yf * yf).sum(0), 1e-3)


def test_conv256_forced_bn_stats(cuda):
    """The 256-row 8-wave conv256 kernel (forced tile 12: 256 x 256, 8 waves), still the route of 3x3 data gradients:
    forward with the BN statistics epilogue against the f32 reference, partial rows summing to the column sums /
    sums of squares."""
    from distributed_tensorflow_amd.ops import conv as C
    from distributed_tensorflow_amd.ops._util import IntOut, call, ptr, stream
    N, H, W, Cin, K = 64, 28, 28, 128, 256
    x = rnd(N, H, W, Cin, dev=cuda)
    w = torch.randn(K, 3, 3, Cin, device=cuda) / math.sqrt(9 * Cin)
    M = N * H * W
    y = torch.empty(N, H, W, K, device=cuda, dtype=BF)
    part = torch.empty(((M + 63) // 64) * 2 * K, dtype=F32, device=cuda)
    ro = IntOut()
    call("dtf_conv_fwd", ptr(x), ptr(w.to(BF)), ptr(y), None, ptr(part), ro.addr, N, H, W, Cin, K, 3, 3, H, W, 1, 1,
         1, 1, 1, 1, 0, 0, 12, stream())
    rows = ro.value
    yr = torch.nn.functional.conv2d(x.float().permute(0, 3, 1, 2), w.to(BF).float().permute(0, 3, 1, 2), padding=1)
    close(y.permute(0, 3, 1, 2).float(), yr, 1e-2)
    p = part[:rows * 2 * K].view(rows, 2 * K).sum(0)
    yf = y.float().reshape(-1, K)
    close(p[:K], yf.sum(0), 1e-3)
    close(p[K:], (yf * yf).sum(0), 1e-3)


@pytest.mark.parametrize("fmt,act", [(0, 0), (1, 0), (1, 2)])
def test_fp8_transposing_quantizer(cuda, fmt, act):
    """dtf_quant_fp8_t: q, q^T, bias-gradient column sums and amax in one pass (e4m3 / e5m2, GELU backward)."""
    from distributed_tensorflow_amd.ops import fp8
    M, N = 256, 192
    x = rnd(M, N, dev=cuda)
    pre = rnd(M, N, dev=cuda) if act else None
    v = x.float()
    if act:
        p = pre.float()
        t = torch.tanh(0.7978845608028654 * (p + 0.044715 * p ** 3))
        v = v * (0.5 * (1 + t) + 0.5 * p * (1 - t * t) * 0.7978845608028654 * (1 + 3 * 0.044715 * p * p))
    fmax = 57344.0 if fmt else 448.0
    scale = (v.abs().max() / fmax).reshape(1)
    amax = torch.zeros(1, device=cuda)
    q, qT, cp = fp8.quantize_t(x, scale, amax, fmt=fmt, pre=pre, act=act, colsums=True)
    dt = torch.float8_e5m2 if fmt else torch.float8_e4m3fn
    dq = q.view(dt).float() * scale
    assert (dq - v).abs().max().item() <= (0.13 if fmt else 0.07) * v.abs().max().item()
    assert torch.equal(qT, q.t().contiguous())
    close(cp.sum(0), v.sum(0), 1e-3)
    assert abs(amax.item() - v.abs().max().item()) <= 1e-6 * v.abs().max().item() + 1e-12


def test_fp8_backward_matches_bf16(cuda):
    """The fp8 backward (e5m2 gradients x e4m3 weights / activations on the scaled MFMA) against the bf16 backward
    of the same fp8 forward (same layer, same delayed scales): dX, dW, db within e5m2 quantization error."""
    from distributed_tensorflow_amd.models.transformer import _Proj
    from distributed_tensorflow_amd.ops import fp8
    torch.manual_seed(0)
    x0 = rnd(512, 256, dev=cuda)
    g = torch.randn(512, 384, device=cuda).to(BF)
    layer = _Proj(384, activation="gelu", fp8=True)
    layer(x0)  # build + bootstrap the activation scale
    outs = []
    for bwd in (False, True):
        fp8._FP8_BWD = bwd
        try:
            layer.kernel.grad = layer.bias.grad = None
            x = x0.clone().requires_grad_(True)
            y = layer(x)
            y.backward(g)
            outs.append((y.float(), x.grad.float(), layer.kernel.grad.float(), layer.bias.grad.float()))
        finally:
            fp8._FP8_BWD = True
    rels = [((a - b).norm() / a.norm()).item() for a, b in zip(outs[0], outs[1])]
    assert rels[0] < 1e-6 and max(rels) < 0.06, rels


@pytest.mark.parametrize("w4", [True, False])
@pytest.mark.parametrize("fmt_a,out_f32,splitk,M,N,K", [(0, False, 1, 256, 128, 256), (1, False, 1, 256, 128, 256),
                                                        (1, False, 1, 1024, 1024, 1024),
                                                        (0, False, 1, 1000, 392, 384),
                                                        (1, True, 1, 256, 128, 512), (1, True, 4, 512, 512, 4096)])
def test_fp8_gemm_formats(cuda, fmt_a, out_f32, splitk, M, N, K, w4):
    """dtf_gemm_fp8_ex: e4m3 / e5m2 A x e4m3 B on the scaled MFMA vs the torch decode of the same bytes; w4: the
    4-wave kernel on v_mfma_scale_f32_32x32x64_f8f6f4 (gemm_w4_fp8.hip, the default), else the 8-wave / 128-row
    kernels on the 16x16x128 form — pinned through the launch counters."""
    from distributed_tensorflow_amd.ops import fp8, _util
    from distributed_tensorflow_amd._native import kernels
    kernels().dtf_fp8_w4_enable(int(w4))
    before = _util.launch_counts()
    try:
        _fp8_gemm_formats(cuda, fmt_a, out_f32, splitk, M, N, K)
    finally:
        kernels().dtf_fp8_w4_enable(-1)
    d = _util.launch_delta(before)
    assert (d["w4f8_256"] + d["w4f8_128"] > 0) == w4, d


def _fp8_gemm_formats(cuda, fmt_a, out_f32, splitk, M, N, K):
    from distributed_tensorflow_amd.ops import fp8
    torch.manual_seed(0)
    da = torch.float8_e5m2 if fmt_a else torch.float8_e4m3fn
    a = (torch.randn(M, K, device=cuda) * 4).to(da)
    b = (torch.randn(N, K, device=cuda) * 4).to(torch.float8_e4m3fn)
    scales = torch.tensor([0.5, 0.25], device=cuda)
    ref = (a.float() @ b.float().t()) * 0.125
    if out_f32:
        out = torch.full((M, N), 1.0, device=cuda)
        fp8.gemm_fp8(a.view(torch.uint8), b.view(torch.uint8), scales, out, fmt_a=fmt_a, out_f32=True, beta=1.0,
                     splitk=splitk)
        ref = ref + 1.0
    else:
        out = torch.empty((M, N), dtype=BF, device=cuda)
        fp8.gemm_fp8(a.view(torch.uint8), b.view(torch.uint8), scales, out, fmt_a=fmt_a)
    close(out, ref, 1e-2)


@pytest.mark.parametrize("bn", [256, 128])
@pytest.mark.parametrize("act", [0, 1, 2])
def test_w4_fp8_epilogue(cuda, bn, act):
    """The 4-wave fp8 kernel's bf16 epilogue (device scales, bias, activation with the pre-activation side output)
    through dtf_gemm_fp8, and its direct entry at both tile widths, vs f32 references of the decoded bytes."""
    from distributed_tensorflow_amd.ops._util import call, ptr, stream, launch_counts, launch_delta
    torch.manual_seed(1)
    M, N, K = 1280, 648, 640
    a = (torch.randn(M, K, device=cuda) * 2).to(torch.float8_e4m3fn)
    b = (torch.randn(N, K, device=cuda) * 2).to(torch.float8_e4m3fn)
    z = a.float() @ b.float().t()
    out = torch.empty((M, N), dtype=F32, device=cuda)
    before = launch_counts()
    call("dtf_gemm_w4_fp8", ptr(a), ptr(b), ptr(out), M, N, K, K, K, N, 0, 1, bn, stream())
    assert launch_delta(before)["w4f8_%d" % bn] == 1
    close(out, z, 1e-4)
    scales = torch.tensor([0.5, 0.125], device=cuda)
    bias = torch.randn(N, device=cuda)
    y = torch.empty((M, N), dtype=BF, device=cuda)
    pre = torch.empty((M, N), dtype=BF, device=cuda)
    call("dtf_gemm_fp8", ptr(a), ptr(b), ptr(y), ptr(pre), ptr(bias), ptr(scales), M, N, K, K, K, N, act, -1, stream())
    p = z * 0.0625 + bias
    close(pre, p, 1e-2)
    ref = torch.relu(p) if act == 1 else torch.nn.functional.gelu(p, approximate="tanh") if act == 2 else p
    close(y, ref, 1e-2)


@pytest.mark.parametrize("ak,bk", [(False, False), (False, True), (True, False), (True, True)])
@pytest.mark.parametrize("M,N,K", [(4096, 1024, 512), (4096, 1096, 384)])
def test_gemm256_narrow_tiles(cuda, ak, bk, M, N, K):
    """256x128 tiles of the pipelined kernel (picked when 256x256 would leave half the chip idle) in all four
    operand layouts vs an fp32 reference."""
    torch.manual_seed(0)
    a = rnd(K, M, dev=cuda) if ak else rnd(M, K, dev=cuda)
    b = rnd(K, N, dev=cuda) if bk else rnd(N, K, dev=cuda)
    out = torch.empty(M, N, dtype=F32, device=cuda)
    from distributed_tensorflow_amd.ops._util import call, ptr, stream
    call("dtf_gemm256_bn", ptr(a), ptr(b), ptr(out), M, N, K, a.stride(0), b.stride(0), N, int(ak), int(bk), 1, 128,
         stream())  # (raises on a non-zero status)
    A = a.float().t() if ak else a.float()
    B = b.float() if bk else b.float().t()
    close(out, A @ B, 2e-2)


@pytest.mark.parametrize("act", ["gelu", "relu"])
def test_dense_pair_fused_activation_backward(cuda, act):
    """FFN1 -> FFN2 with FFN1's activation backward fused into FFN2's data-gradient GEMM (dtf_gemm_dact) gives the
    same gradients as the unfused pair (bitwise: the product is rounded to bf16 before act', as dtf_act does)."""
    from distributed_tensorflow_amd.ops import linalg as LA
    torch.manual_seed(0)
    x0 = rnd(512, 256, dev=cuda)
    w1 = (torch.randn(1024, 256, device=cuda) * 0.05).requires_grad_(True)
    b1 = torch.zeros(1024, device=cuda, requires_grad=True)
    w2 = (torch.randn(256, 1024, device=cuda) * 0.05).requires_grad_(True)
    g = rnd(512, 256, dev=cuda)
    from distributed_tensorflow_amd.ops._util import launch_counts, launch_delta
    res = []
    for fuse in (False, True):
        before = launch_counts()
        x = x0.clone().requires_grad_(True)
        h = LA.dense(x, w1, b1, act=act, tag_act=fuse)
        y = LA.dense(h, w2, None)
        y.backward(g)
        # the fused run reaches dtf_gemm_dact (activation backward in FFN2's data-gradient epilogue), the other not
        assert launch_delta(before)["gemm_dact"] == (1 if fuse else 0)
        res.append((x.grad.clone(), w1.grad.clone(), b1.grad.clone(), w2.grad.clone()))
        for t in (w1, b1, w2):
            t.grad = None
    for a, b in zip(res[0], res[1]):
        assert torch.equal(a, b)


def test_dropout_keep_rate_and_scale(cuda):
    """Elementwise dropout (16-bit uniforms from chunk hashes): realised keep rate ~= keep, kept values scaled by the
    exact inverse of the 16-bit threshold, fresh masks for different seeds."""
    x = torch.ones(1 << 20, device=cuda).to(BF)
    y1 = ops.dropout(x, 0.1, training=True, seed=7).float()
    y2 = ops.dropout(x, 0.1, training=True, seed=8).float()
    kept = (y1 != 0).float().mean().item()
    assert abs(kept - 0.9) < 0.003, kept
    vals = y1[y1 != 0]
    assert torch.allclose(vals, torch.full_like(vals, 65536.0 / round(0.9 * 65536)).to(BF).float())
    assert ((y1 != 0) != (y2 != 0)).float().mean().item() > 0.1


@pytest.mark.gpu
@pytest.mark.parametrize("M,N,K", [(4096, 768, 2304), (2048, 1024, 4096), (1000, 776, 512)])
def test_gemm_beta_bf16_equals_gemm_then_add(cuda, M, N, K):
    """C = A.B^T + C for bf16 C (the residual-gradient join of a data-gradient GEMM, ops.linalg.dense_dgrad with
    acc): bit-identical to the plain GEMM followed by an f32 add rounded once — on the 256x256 kernel's staged
    store pass as on the 128x128 kernels."""
    torch.manual_seed(0)
    a = torch.randn(M, K, device=cuda).to(torch.bfloat16)
    w = torch.randn(K, N, device=cuda).to(torch.bfloat16)  # K-outer B, as a data gradient reads W
    c0 = torch.randn(M, N, device=cuda).to(torch.bfloat16)
    prod = ops.gemm(a, w, b_kouter=True)
    ref = (prod.float() + c0.float()).to(torch.bfloat16)
    out = c0.clone()
    ops.gemm(a, w, b_kouter=True, out=out, beta=1.0)
    assert torch.equal(out, ref)
    close(prod, a.float() @ w.float(), 2e-2)


@pytest.mark.gpu
@pytest.mark.parametrize("T,W,stride", [(6272, 128, 128), (1568, 512, 512), (392, 1024, 1024), (100, 96, 100),
                                        (45, 2048, 2048), (700, 4096, 4096)])
def test_row_reductions_large(cuda, T, W, stride):
    """Deterministic partial-row reductions at the sizes the BN statistics and bias/LN gradients produce: the
    grouping pass (dtf_group_rows_once: <= 32 leader rows written over each group's first row) and the full
    sum (dtf_sum_rows, with accumulate) against an f64 sum."""
    import ctypes
    torch.manual_seed(0)
    rows = torch.randn(T, stride, device=cuda)
    ref = rows[:, :W].double().sum(0)
    r2 = rows.clone()
    out_stride = ctypes.c_long(0)
    n = _util.K().dtf_group_rows_once(_util.ptr(r2), stride, T, W, 32, ctypes.byref(out_stride), _util.stream())
    s = out_stride.value
    lead = torch.stack([r2.view(-1)[i * s:i * s + W] for i in range(n)]).double().sum(0)
    torch.testing.assert_close(lead, ref, rtol=1e-5, atol=1e-3)
    out = torch.ones(W, device=cuda)
    _util.K().dtf_sum_rows(_util.ptr(rows), stride, T, W, _util.ptr(out), 1, _util.stream())
    torch.testing.assert_close(out.double(), ref + 1.0, rtol=1e-5, atol=1e-3)


@pytest.mark.parametrize("T,M,N", [(4096, 768, 1024), (8192, 1024, 4096), (1024, 264, 136)])
def test_dense_wgrad_bias_fused(cuda, T, M, N):
    """dW += dZ^T X and db += colsum(dZ) in one 4-wave GEMM launch (the bias gradient from the dZ fragments by
    v_dot2c against 1.0, GemmArgs::rowsum) vs the weight-gradient GEMM + the column-sum pass: dW bit for bit (same
    kernel, split plan and slab reduction), db to f32 rounding; both vs the f32 reference."""
    from distributed_tensorflow_amd.ops import linalg as LA
    from distributed_tensorflow_amd.ops._util import launch_counts, launch_delta
    torch.manual_seed(0)
    dz = rnd(T, M, dev=cuda)
    x = rnd(T, N, dev=cuda)
    w0 = torch.randn(M, N, device=cuda)
    b0 = torch.randn(M, device=cuda)
    tw, tb = w0.clone(), b0.clone()
    before = launch_counts()
    assert LA.dense_wgrad_bias(dz, x, tw, tb)
    d = launch_delta(before)
    assert d["w4_256"] + d["w4_128"] == 1, d
    uw, ub = w0.clone(), b0.clone()
    LA.dense_wgrad(dz, x, out=uw)
    LA.colsum(dz, out=ub, accumulate=True)
    torch.cuda.synchronize()
    assert torch.equal(tw, uw)
    torch.testing.assert_close(tb, ub, rtol=1e-5, atol=1e-3)
    close(tw, w0 + dz.float().t() @ x.float(), 1e-3)
    close(tb, b0 + dz.float().sum(0), 1e-4)



@pytest.mark.parametrize("case", [(4, 14, 14, 256, 256), (3, 9, 11, 512, 128), (2, 7, 7, 512, 512)])
@pytest.mark.parametrize("with_bn", [True, False])
def test_conv_dgrad_w4_gather_bn_stats(cuda, case, with_bn):
    """Stride-1 3x3 data gradients into >= 256 channels take the 4-wave kernel with the dY gather loader
    (gemm_w4.h W4Gather<OP_DGRAD_T>): dX against the f32 autograd reference on odd / partial-tile shapes, and with a
    BatchNorm(+ReLU) input the BN-backward partial rows (sum dz, sum dz * (x - mean), dz = dX * mask) of the stored
    values; launch-counted."""
    from distributed_tensorflow_amd.ops import conv as C
    from distributed_tensorflow_amd.ops._util import IntOut, call, crsk_shadow, launch_counts, launch_delta, ptr, \
        stream, workspace
    N, H, W, Cin, K = case
    R = S = 3
    dy = rnd(N, H, W, K, dev=cuda)
    w = torch.randn(K, R, S, Cin, device=cuda) / math.sqrt(R * S * Cin)
    x = rnd(N, H, W, Cin, dev=cuda)
    g = C._geom(x, w, (1, 1), (1, 1), (1, 1))
    M = N * H * W
    yc = rnd(N, H, W, Cin, dev=cuda)
    mask = torch.rand(M * Cin, device=cuda) > 0.4
    bits = (mask.view(-1, 8).to(torch.uint8) << torch.arange(8, device=cuda, dtype=torch.uint8)).sum(1).to(torch.uint8)
    mean = torch.randn(Cin, device=cuda) * 0.1
    dx = torch.empty(N, H, W, Cin, device=cuda, dtype=BF)
    part = torch.empty(((M + 63) // 64 + 1) * 2 * Cin, dtype=torch.float32, device=cuda)
    rows = IntOut()
    ws = workspace(cuda)
    wc = crsk_shadow(w, K, R * S, Cin)
    before = launch_counts()
    bn = (ptr(yc), ptr(bits), ptr(mean), ptr(part), rows.addr) if with_bn else (None, None, None, None, None)
    call("dtf_conv_dgrad", ptr(dy), ptr(wc), ptr(dx), N, H, W, Cin, K, R, S, g[7], g[8], 1, 1, 1, 1, 1, 1, 0,
         0.0, -1, ptr(ws), 2 * ws.numel(), *bn, None, stream())
    torch.cuda.synchronize()
    d = launch_delta(before)
    assert d["w4_256"] + d["w4_128"] == 1, d
    xr = torch.zeros(N, Cin, H, W, device=cuda, requires_grad=True)
    torch.nn.functional.conv2d(xr, w.to(BF).float().permute(0, 3, 1, 2), padding=1).backward(
        dy.float().permute(0, 3, 1, 2))
    close(dx.permute(0, 3, 1, 2).float(), xr.grad, 1e-2)
    if with_bn:
        T = rows.value
        assert T == (M + 255) // 256
        p = part[:T * 2 * Cin].view(T, 2 * Cin).sum(0)
        dz = dx.float().reshape(M, Cin) * mask.view(M, Cin).float()
        close(p[:Cin], dz.sum(0), 1e-3)
        close(p[Cin:], (dz * (yc.float().reshape(M, Cin) - mean)).sum(0), 1e-3)



@pytest.mark.parametrize("T,D,V", [(65536, 768, 2), (4099, 1024, 3), (1001, 200, 1), (777, 2048, 4), (3000, 256, 9),
                                   (2050, 520, 16)])
def test_embed_bwd_small_table(cuda, T, D, V):
    """Gradient of a small embedding table (BERT's token types): out[v] (+)= sum of dy over the tokens of type v —
    register accumulators per wave (elementwise.hip embed_bwd_regs_kernel, 4 table rows per launch); vs the f32
    reference, accumulating, and the same bits on a second run (no atomics)."""
    from distributed_tensorflow_amd.ops._util import call, ptr, stream, workspace
    torch.manual_seed(0)
    dy = rnd(T, D, dev=cuda)
    idx = torch.randint(0, V, (T,), device=cuda)
    ws = workspace(cuda)
    base = torch.randn(V, D, device=cuda)
    outs = []
    for _ in range(2):
        out = base.clone()
        call("dtf_embed_bwd_small", ptr(dy), ptr(idx), ptr(out), T, D, V, 1, ptr(ws), ws.numel(), stream())
        outs.append(out)
    torch.cuda.synchronize()
    ref = base + torch.zeros(V, D, device=cuda).index_add_(0, idx, dy.float())
    close(outs[0], ref, 1e-4)
    assert torch.equal(outs[0], outs[1])
