"""Producer-side fp8 quantization (ops.fp8 DTF_FP8_FUSE, gemm256.hip q8 epilogue outputs): the GEMM epilogue
writes the next fp8 layer's operand (row-major + transposed, delayed scaling) or the previous layer's e5m2 gradient
(activation backward applied, transposed, bias-gradient column sums) instead of a bf16 tensor + a quantize pass.
Checked against the unfused pair (dtf_gemm_fp8_ex + dtf_quant_fp8_t2) on the same bytes."""
import pytest
import torch

from distributed_tensorflow_amd.ops import fp8
from distributed_tensorflow_amd.ops._util import K, ptr, stream

pytestmark = pytest.mark.gpu
BF = torch.bfloat16


@pytest.fixture(scope="module")
def cuda():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


def _q8(a, b, scales, C, M, N, Kd, *, fmt_a, act=0, aux=None, bias=None, dact_src=None, dact=0, q8=None, q8T=None,
        q8col=None, q8fmt=0, buf=None):
    """buf: [scale, amax, amax_prev, used, used2] f32 slots"""
    return K().dtf_gemm_fp8_q8(ptr(a), ptr(b), ptr(C), ptr(aux), ptr(bias), ptr(scales), M, N, Kd, a.stride(0),
                               b.stride(0), act, fmt_a, ptr(dact_src), dact, None, ptr(q8), ptr(q8T), ptr(q8col),
                               q8fmt, ptr(buf[0:1]), ptr(buf[1:2]), ptr(buf[2:3]), ptr(buf[3:4]), ptr(buf[4:5]),
                               stream())


@pytest.fixture(params=[0, 1], ids=["q8-gemm256", "q8-w4"])
def q8_kernel(request):
    """The producer-quantizing GEMM on the 8-wave gemm256 epilogue (the default for q8 GEMMs) or on the 4-wave fp8
    kernel's (gemm_w4_fp8.hip w8_epilogue), pinned through the launch counters. The plain reference GEMM of a test runs
    on the same kernel family (its accumulation order is part of what is compared bit for bit)."""
    from distributed_tensorflow_amd.ops._util import launch_counts, launch_delta
    K().dtf_fp8_w4_enable(request.param)
    before = launch_counts()
    yield request.param
    K().dtf_fp8_w4_enable(-1)
    d = launch_delta(before)
    if request.param == 1:
        assert d["w4f8_256"] + d["w4f8_128"] > 0 and d["gemm256_fp8"] == 0, d
    else:
        assert d["gemm256_fp8"] > 0, d


@pytest.mark.parametrize("M,N,Kd", [(512, 1024, 256), (768, 512, 384)])
def test_q8_forward_epilogue_matches_quantize_pass(cuda, M, N, Kd, q8_kernel):
    """GELU projection: the fp8 copies (q, q^T), the delayed scale it used and the recorded amax are bit-identical
    to quantizing the bf16 output of the same GEMM with the transposing quantizer; the pre-activation side output is
    unchanged and no bf16 output is written."""
    torch.manual_seed(1)
    a = (torch.randn(M, Kd, device=cuda) * 2).to(torch.float8_e4m3fn).view(torch.uint8)
    b = (torch.randn(N, Kd, device=cuda) * 2).to(torch.float8_e4m3fn).view(torch.uint8)
    scales = torch.tensor([0.05, 0.02], device=cuda)
    bias = torch.randn(N, device=cuda) * 0.1
    y = torch.empty(M, N, dtype=BF, device=cuda)
    pre = torch.empty(M, N, dtype=BF, device=cuda)
    fp8.gemm_fp8(a, b, scales, y, bias=bias, act=2, aux=pre)
    amax_prev = y.float().abs().max().reshape(1) * 0.9  # "last step's" amax: sets this step's scale
    ref_buf = torch.tensor([1.0, 0.0, amax_prev.item(), 0.0, 0.0], device=cuda)
    q_ref, qT_ref, _ = fp8.quantize_t(y, ref_buf[0:1], ref_buf[1:2], amax_prev=ref_buf[2:3], scale_used=ref_buf[3:4],
                                      scale_used2=ref_buf[4:5])
    buf = torch.tensor([1.0, 0.0, amax_prev.item(), 0.0, 0.0], device=cuda)
    q = torch.empty(M, N, dtype=torch.uint8, device=cuda)
    qT = torch.empty(N, M, dtype=torch.uint8, device=cuda)
    pre2 = torch.empty(M, N, dtype=BF, device=cuda)
    rc = _q8(a, b, scales, None, M, N, Kd, fmt_a=0, act=2, aux=pre2, bias=bias, q8=q, q8T=qT, q8fmt=0, buf=buf)
    assert rc == 0, rc
    torch.cuda.synchronize()
    assert torch.equal(pre2, pre)
    assert torch.equal(q, q_ref)
    assert torch.equal(qT, qT_ref)
    assert torch.equal(buf[1], ref_buf[1]) and buf[1].item() > 0  # amax
    assert torch.equal(buf[3:5], ref_buf[3:5]) and buf[3].item() > 0  # scale used (both slots)


def test_q8_backward_epilogue_gelu_grad(cuda, q8_kernel):
    """Data-gradient GEMM (e5m2 x e4m3) whose output is the gradient of a GELU: e5m2 copy of dZ = (dY W) * gelu'(pre)
    with its transpose and per-128-row column sums vs the bf16 GEMM + the transposing quantizer (which applies the
    GELU backward in f32; the fused epilogue rounds dZ to bf16 first: bytes may differ by one e5m2 step)."""
    torch.manual_seed(2)
    M, N, Kd = 512, 768, 256
    a = (torch.randn(M, Kd, device=cuda) * 4).to(torch.float8_e5m2).view(torch.uint8)
    b = (torch.randn(N, Kd, device=cuda) * 2).to(torch.float8_e4m3fn).view(torch.uint8)
    scales = torch.tensor([0.01, 0.03], device=cuda)
    pre = (torch.randn(M, N, device=cuda) * 2).to(BF)
    y = torch.empty(M, N, dtype=BF, device=cuda)
    fp8.gemm_fp8(a, b, scales, y, fmt_a=1)
    ref_buf = torch.tensor([1.0, 0.0, 0.0, 0.0, 0.0], device=cuda)
    ref_buf[2] = y.float().abs().max() * 1.1
    q_ref, qT_ref, cp_ref = fp8.quantize_t(y, ref_buf[0:1], ref_buf[1:2], fmt=1, pre=pre, act=2, colsums=True,
                                           amax_prev=ref_buf[2:3], scale_used=ref_buf[3:4])
    buf = ref_buf.clone()
    buf[1] = 0.0
    q = torch.empty(M, N, dtype=torch.uint8, device=cuda)
    qT = torch.empty(N, M, dtype=torch.uint8, device=cuda)
    cp = torch.empty(M // 128, N, dtype=torch.float32, device=cuda)
    rc = _q8(a, b, scales, None, M, N, Kd, fmt_a=1, dact_src=pre, dact=2, q8=q, q8T=qT, q8col=cp, q8fmt=1, buf=buf)
    assert rc == 0, rc
    torch.cuda.synchronize()
    assert torch.equal(qT, q.t().contiguous())
    sc = buf[3].item()
    assert sc == ref_buf[3].item() and sc > 0
    dq = q.view(torch.float8_e5m2).float() * sc
    dq_ref = q_ref.view(torch.float8_e5m2).float() * sc
    # at most one e5m2 step apart (2 mantissa bits: a step is <= 1/4 of the value), subnormals aside
    assert bool(((dq - dq_ref).abs() <= 0.25 * torch.maximum(dq.abs(), dq_ref.abs()) + 2.0 ** -16 * sc).all())
    assert (q == q_ref).float().mean().item() > 0.97
    torch.testing.assert_close(cp.sum(0), cp_ref.sum(0), rtol=2e-2, atol=2e-2 * cp_ref.abs().max().item())
    assert abs(buf[1].item() - ref_buf[1].item()) <= 0.02 * ref_buf[1].item()


def test_q8_rejects_unaligned_rows(cuda):
    """M not a multiple of 256: -6 and nothing launched (the caller keeps the bf16 output + quantize pass)."""
    a = torch.zeros(200, 128, dtype=torch.uint8, device=cuda)
    b = torch.zeros(256, 128, dtype=torch.uint8, device=cuda)
    buf = torch.ones(5, device=cuda)
    q = torch.empty(200, 256, dtype=torch.uint8, device=cuda)
    assert _q8(a, b, torch.ones(2, device=cuda), None, 200, 256, 128, fmt_a=0, q8=q, buf=buf) == -6


def test_gpt2_fused_fp8_path_matches_unfused(cuda, monkeypatch):
    """Tiny GPT-2 (fp8 projections), two forward/backward passes (the first bootstraps the delayed scales): with
    DTF_FP8_FUSE the FFN1 epilogue writes FFN2's e4m3 operand and FFN2's data-gradient epilogue writes FFN1's e5m2
    gradient (2 fused GEMMs per block and pass, 2 fewer quantize passes) — the loss matches the unfused path and
    every gradient agrees within e5m2 rounding."""
    from distributed_tensorflow_amd.keras import initializers
    from distributed_tensorflow_amd.models.transformer import GPT2
    from distributed_tensorflow_amd.ops import _util
    g = torch.Generator().manual_seed(5)
    V, S, B = 512, 128, 4
    ids = torch.randint(0, V, (B, S), generator=g).to(cuda)
    tgt = torch.roll(ids, -1, 1)
    seen = []
    real_call = _util.call

    def spy(name, *args):
        seen.append(name)
        return real_call(name, *args)

    monkeypatch.setattr(fp8, "call", spy)

    def run(fuse, use_fp8=True):
        monkeypatch.setattr(fp8, "_FUSE", fuse)
        initializers.set_seed(21)
        model = GPT2(vocab=V, ctx=S, hidden=256, layers=2, heads=4, dropout=0.0, fp8=use_fp8)
        out = None
        for it in range(2):
            seen.clear()
            for p in model.trainable_weights:
                p.grad = None
            logits = model(ids, training=True)
            loss = torch.nn.functional.cross_entropy(logits.float().reshape(-1, logits.shape[-1])[:, :V],
                                                     tgt.reshape(-1))
            loss.backward()
            torch.cuda.synchronize()
            out = (loss.item(), {i: p.grad.float().clone()
                                 for i, p in enumerate(model.trainable_weights) if p.grad is not None},
                   seen.count("dtf_quant_fp8_t2"))
        return out

    lf, gf, nq_f = run(True)
    lu, gu, nq_u = run(False)
    _, gb, _ = run(False, use_fp8=False)
    assert abs(lf - lu) <= 1e-4 * abs(lu), (lf, lu)
    assert nq_u - nq_f == 2 * 2, (nq_u, nq_f)  # 2 blocks x (FFN2 input + FFN1 gradient)
    assert gf.keys() == gu.keys() == gb.keys()

    def rel(a, b):
        return ((a - b).norm() / (b.norm() + 1e-12)).item()
    # the fused path is as close to the bf16 gradients as the unfused fp8 path (both carry e5m2 gradient noise)
    bad = {k: (rel(gf[k], gb[k]), rel(gu[k], gb[k])) for k in gb
           if rel(gf[k], gb[k]) > 1.25 * rel(gu[k], gb[k]) + 0.01}
    assert not bad, bad

