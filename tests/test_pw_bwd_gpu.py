"""Fused data + weight gradient of the ResNet-50 stage-1 channel-reducing 1x1 conv (csrc/kernels/pwbwd.hip,
dtf_pw_conv_bwd): one pass over dY gives dX (+ the BatchNorm-backward partial rows of dX) and dW.

dX must equal, BITWISE, the separate data-gradient GEMM (same k order per MFMA chain); dW and the partial sums agree
with the separate kernels to f32 summation order, and all three with a plain PyTorch fp32 reference. At block level
the gradients of three stage-1 bottlenecks with the fused path on and off agree to that summation order. The
reference's op is the gradient of the Conv2D the ResNet-50 trainer builds (trainer/task.py:62-71)."""
import ctypes

import pytest
import torch

from distributed_tensorflow_amd.ops import conv as OC
from distributed_tensorflow_amd.ops._util import call, ptr, stream

pytestmark = pytest.mark.gpu

BF = torch.bfloat16
F32 = torch.float32


def _bits(b):
    M, N = b.shape
    w = (1 << torch.arange(8, device=b.device, dtype=torch.int32))
    return (b.view(M, N // 8, 8).to(torch.int32) * w).sum(-1).to(torch.uint8).view(-1)


@pytest.mark.parametrize("P", [16384, 50000, 200003])
@pytest.mark.parametrize("with_bn", [False, True])
def test_pw_bwd_matches_separate_kernels(cuda, P, with_bn):
    K, C = 256, 64
    g = torch.Generator(device="cpu").manual_seed(P + int(with_bn))
    dy = torch.randn(P, K, generator=g).to(BF).to(cuda)
    x = torch.relu(torch.randn(P, C, generator=g)).to(BF).to(cuda)
    wck = (torch.randn(C, K, generator=g) * K ** -0.5).to(BF).to(cuda)  # [C][1][1][K]
    dw0 = torch.randn(K, C, generator=g).to(cuda)
    bnx = _bits(torch.rand(P, C, generator=g) > 0.5) if with_bn else None
    bn = (torch.randn(P, C, generator=g).to(BF).to(cuda), bnx.to(cuda),
          (torch.randn(C, generator=g) * 0.1).to(cuda)) if with_bn else (None, None, None)
    ws = torch.empty(32 << 20, dtype=F32, device=cuda)
    # fused
    dx = torch.full((P, C), float("nan"), dtype=BF, device=cuda)
    dw = dw0.clone()
    part = torch.full((256 * 2 * C,), float("nan"), device=cuda) if with_bn else None
    rows = ctypes.c_int(0)
    call("dtf_pw_conv_bwd", ptr(dy), ptr(x), ptr(wck), ptr(dx), ptr(dw), 1, ptr(bn[0]), ptr(bn[1]), ptr(bn[2]),
         ptr(part), ctypes.addressof(rows), ptr(ws), ws.numel(), P, K, C, stream())
    # separate: data gradient (general tile) and weight gradient
    dx2 = torch.empty(P, C, dtype=BF, device=cuda)
    part2 = torch.empty((((P + 63) // 64) + 1) * 2 * C, device=cuda) if with_bn else None
    rows2 = ctypes.c_int(0)
    call("dtf_set_pw_dgrad", 0)
    try:
        call("dtf_conv_dgrad_x", ptr(dy), ptr(wck), ptr(dx2), P, 1, 1, C, K, 1, 1, 1, 1, 1, 1, 0, 0, 1, 1, 0.0,
             ptr(ws), 16, ptr(bn[0]), ptr(bn[1]), ptr(bn[2]), ptr(part2),
             ctypes.addressof(rows2) if with_bn else None, None, None, None, None, stream())
    finally:
        call("dtf_set_pw_dgrad", 1)
    dw2 = dw0.clone()
    call("dtf_conv_wgrad", ptr(x), ptr(dy), ptr(dw2), P, 1, 1, C, K, 1, 1, 1, 1, 1, 1, 0, 0, 1, 1, 1, 0, -1,
         ptr(ws), ws.numel(), stream())
    torch.cuda.synchronize()
    assert torch.equal(dx.view(torch.int16), dx2.view(torch.int16)), "dX differs from the separate dgrad"
    ref_dx = dy.float() @ wck.float().t()
    assert torch.allclose(dx.float(), ref_dx, atol=3e-2, rtol=2e-2)
    ref_dw = dw0 + dy.float().t() @ x.float()
    scale = ref_dw.abs().max().item()
    assert (dw - ref_dw).abs().max().item() <= 1e-4 * scale + 1e-3
    assert (dw - dw2).abs().max().item() <= 1e-4 * scale + 1e-3
    if with_bn:
        assert rows.value == 256
        s1 = part.view(256, 2 * C).sum(0)
        s2 = part2[: rows2.value * 2 * C].view(rows2.value, 2 * C).sum(0)
        sc = s2.abs().max().item() + 1.0
        assert torch.allclose(s1, s2, atol=1e-4 * sc, rtol=1e-4)


@pytest.mark.parametrize("P", [8192, 100003])
def test_pw_bwd_bn_stage2_matches_separate_kernels(cuda, P):
    """Stage-2 shape (K_out 512 from C_in 128: two column blocks per 32-pixel slot): dX bitwise the apply pass +
    general data-gradient tile, dW and the BN partial sums to f32 summation order, against fp32 references too."""
    K, C = 512, 128
    g = torch.Generator(device="cpu").manual_seed(P + 1)
    dout = torch.randn(P, K, generator=g).to(BF).to(cuda)
    y = torch.randn(P, K, generator=g).to(BF).to(cuda)
    ym = _bits(torch.rand(P, K, generator=g) > 0.3).to(cuda)
    coef = torch.cat([torch.rand(K, generator=g) + 0.5, torch.randn(K, generator=g) * 0.1,
                      torch.randn(K, generator=g) * 0.01]).to(cuda)
    x = torch.relu(torch.randn(P, C, generator=g)).to(BF).to(cuda)
    wck = (torch.randn(C, K, generator=g) * K ** -0.5).to(BF).to(cuda)
    bn = (torch.randn(P, C, generator=g).to(BF).to(cuda), _bits(torch.rand(P, C, generator=g) > 0.5).to(cuda),
          (torch.randn(C, generator=g) * 0.1).to(cuda))
    ws = torch.empty(32 << 20, dtype=F32, device=cuda)
    dx = torch.full((P, C), float("nan"), dtype=BF, device=cuda)
    dw0 = torch.randn(K, C, generator=g).to(cuda)
    dw = dw0.clone()
    part = torch.full((256 * 2 * C,), float("nan"), device=cuda)
    rows = ctypes.c_int(0)
    call("dtf_pw_conv_bwd_bn", ptr(dout), ptr(y), ptr(ym), ptr(coef), ptr(x), ptr(wck), ptr(dx), ptr(dw), 1,
         ptr(bn[0]), ptr(bn[1]), ptr(bn[2]), ptr(part), ctypes.addressof(rows), ptr(ws), ws.numel(), P, K, C,
         None, None, None, None, None, stream())
    dyc = torch.empty(P, K, dtype=BF, device=cuda)
    call("dtf_bn_bwd_apply_coef", ptr(dout), ptr(ym), ptr(y), P, K, ptr(dyc), None, ptr(coef), None, None, None,
         None, stream())
    dx2 = torch.empty(P, C, dtype=BF, device=cuda)
    part2 = torch.empty((((P + 63) // 64) + 1) * 2 * C, device=cuda)
    rows2 = ctypes.c_int(0)
    call("dtf_set_pw_dgrad", 0)
    try:
        call("dtf_conv_dgrad_x", ptr(dyc), ptr(wck), ptr(dx2), P, 1, 1, C, K, 1, 1, 1, 1, 1, 1, 0, 0, 1, 1, 0.0,
             ptr(ws), 16, ptr(bn[0]), ptr(bn[1]), ptr(bn[2]), ptr(part2), ctypes.addressof(rows2), None, None,
             None, None, stream())
    finally:
        call("dtf_set_pw_dgrad", 1)
    torch.cuda.synchronize()
    assert rows.value == 128
    ref_dx = dyc.float() @ wck.float().t()
    assert torch.allclose(dx.float(), ref_dx, atol=3e-2, rtol=2e-2)
    nbad = (dx.view(torch.int16) != dx2.view(torch.int16)).sum().item()
    assert nbad == 0, f"{nbad} dX elements differ from the general tile"
    ref_dw = dw0 + dyc.float().t() @ x.float()
    scale = ref_dw.abs().max().item()
    assert (dw - ref_dw).abs().max().item() <= 1e-4 * scale + 1e-3
    s1 = part[: rows.value * 2 * C].view(rows.value, 2 * C).sum(0)
    s2 = part2[: rows2.value * 2 * C].view(rows2.value, 2 * C).sum(0)
    sc = s2.abs().max().item() + 1.0
    assert torch.allclose(s1, s2, atol=1e-4 * sc, rtol=1e-4)


@pytest.mark.parametrize("P", [16384, 200003])
def test_pw_bwd_bn_matches_apply_then_fused(cuda, P):
    """dtf_pw_conv_bwd_bn (dY computed per tile from dout, y, the ReLU bits and the BN-backward coefficients) equals
    the standalone apply pass (dtf_bn_bwd_apply_coef) followed by dtf_pw_conv_bwd: dX bitwise, dW and the partials
    to f32 summation order."""
    K, C = 256, 64
    g = torch.Generator(device="cpu").manual_seed(P)
    dout = torch.randn(P, K, generator=g).to(BF).to(cuda)
    y = torch.randn(P, K, generator=g).to(BF).to(cuda)
    ym = _bits(torch.rand(P, K, generator=g) > 0.3).to(cuda)
    coef = torch.cat([torch.rand(K, generator=g) + 0.5, torch.randn(K, generator=g) * 0.1,
                      torch.randn(K, generator=g) * 0.01]).to(cuda)
    x = torch.relu(torch.randn(P, C, generator=g)).to(BF).to(cuda)
    wck = (torch.randn(C, K, generator=g) * K ** -0.5).to(BF).to(cuda)
    bn = (torch.randn(P, C, generator=g).to(BF).to(cuda), _bits(torch.rand(P, C, generator=g) > 0.5).to(cuda),
          (torch.randn(C, generator=g) * 0.1).to(cuda))
    ws = torch.empty(32 << 20, dtype=F32, device=cuda)
    dx = torch.full((P, C), float("nan"), dtype=BF, device=cuda)
    dw = torch.zeros(K, C, device=cuda)
    part = torch.full((256 * 2 * C,), float("nan"), device=cuda)
    rows = ctypes.c_int(0)
    call("dtf_pw_conv_bwd_bn", ptr(dout), ptr(y), ptr(ym), ptr(coef), ptr(x), ptr(wck), ptr(dx), ptr(dw), 1,
         ptr(bn[0]), ptr(bn[1]), ptr(bn[2]), ptr(part), ctypes.addressof(rows), ptr(ws), ws.numel(), P, K, C,
         None, None, None, None, None, stream())
    dyc = torch.empty(P, K, dtype=BF, device=cuda)
    call("dtf_bn_bwd_apply_coef", ptr(dout), ptr(ym), ptr(y), P, K, ptr(dyc), None, ptr(coef), None, None, None,
         None, stream())
    dx2 = torch.full((P, C), float("nan"), dtype=BF, device=cuda)
    dw2 = torch.zeros(K, C, device=cuda)
    part2 = torch.full((256 * 2 * C,), float("nan"), device=cuda)
    rows2 = ctypes.c_int(0)
    call("dtf_pw_conv_bwd", ptr(dyc), ptr(x), ptr(wck), ptr(dx2), ptr(dw2), 1, ptr(bn[0]), ptr(bn[1]), ptr(bn[2]),
         ptr(part2), ctypes.addressof(rows2), ptr(ws), ws.numel(), P, K, C, stream())
    torch.cuda.synchronize()
    assert torch.equal(dx.view(torch.int16), dx2.view(torch.int16))
    assert torch.equal(dw, dw2)  # same dY bits, same kernel structure and reduction order
    assert torch.equal(part, part2)
    # and the dY the kernel used is the fp32 formula
    bits = ((ym.view(-1, 1) >> torch.arange(8, device=cuda, dtype=torch.uint8)) & 1).view(P, K).float()
    ref = (coef[:K] * dout.float() * bits + coef[K:2 * K] * y.float() + coef[2 * K:]).to(BF)
    assert (ref.float() - dyc.float()).abs().max().item() <= 1e-2 * ref.float().abs().max().item()


@pytest.mark.parametrize("level", [1, 2, 3, 4])
def test_pw_bwd_block_gradients(cuda, monkeypatch, level):
    """Three stage-1 bottlenecks trained the framework's way (arena gradients, direct accumulation). Level 1: every c3
    and the stride-1 projection take the fused data + weight gradient; level 2: the middle block's c3 (identity
    block whose BN-backward reduction its consumer already took), the projection block's c3 (with the shortcut BN
    reduction) and its stride-1 projection also fold the BatchNorm backward in. Gradients agree
    with the unfused path to f32 summation order. Level 3: the identity blocks' c3 outputs are not stored; the middle
    block's fold recomputes y per tile, the last block's c1 data gradient recomputes its BN input, the last c3
    (no fused reduction: the loss consumes it) materialises it."""
    from distributed_tensorflow_amd.keras import initializers
    from distributed_tensorflow_amd.models import resnet as R
    from distributed_tensorflow_amd.ops._util import direct_grads
    from distributed_tensorflow_amd.variables import ParamArena
    g = torch.Generator().manual_seed(13)
    x = torch.randn(64, 16, 16, 64, generator=g).to(cuda).to(BF)
    runs = {}
    seen = {}
    real_call = OC.call

    def spy(name, *args):
        seen[name] = seen.get(name, 0) + 1
        return real_call(name, *args)

    monkeypatch.setattr(OC, "call", spy)
    for lv in (0, level):
        monkeypatch.setattr(OC, "_FUSED_PW_BWD", lv)
        initializers.set_seed(3)
        blocks = [R.Bottleneck(64, stride=1, project=True), R.Bottleneck(64), R.Bottleneck(64)]
        with torch.no_grad():
            h = x
            for b in blocks:
                h = b(h, training=False)
        params = [w for b in blocks for w in b.trainable_weights]
        arena = ParamArena(params, device=cuda)
        seen.clear()
        xx = x.clone().requires_grad_(True)
        h = xx
        for b in blocks:
            h = b(h, training=True)
        loss = (h.float() * torch.linspace(-1, 1, h.shape[-1], device=cuda)).square().mean()
        with direct_grads():
            loss.backward()
        torch.cuda.synchronize()
        runs[lv] = [xx.grad.float(), arena.grad.clone()]
        want = {0: (0, 0), 1: (4, 0), 2: (1, 3), 3: (1, 3), 4: (1, 3)}[lv]
        assert (seen.get("dtf_pw_conv_bwd", 0), seen.get("dtf_pw_conv_bwd_bn", 0)) == want, seen
    for a, b in zip(runs[0], runs[level]):
        assert torch.isfinite(b).all()
        err = (a - b).norm().item() / (a.norm().item() + 1e-12)
        assert err < 1e-2, err


def test_pw_bwd_bn_stage2_block_gradients(cuda, monkeypatch):
    """Stage-2 bottlenecks (stride-2 projection block + two identity blocks, width 128): the middle block's c3 takes
    the BatchNorm-folded fused path; gradients agree with the unfused path to f32 summation order."""
    from distributed_tensorflow_amd.keras import initializers
    from distributed_tensorflow_amd.models import resnet as R
    from distributed_tensorflow_amd.ops._util import direct_grads
    from distributed_tensorflow_amd.variables import ParamArena
    g = torch.Generator().manual_seed(17)
    x = torch.randn(32, 32, 32, 256, generator=g).to(cuda).to(BF)
    runs = {}
    seen = {}
    real_call = OC.call

    def spy(name, *args):
        seen[name] = seen.get(name, 0) + 1
        return real_call(name, *args)

    monkeypatch.setattr(OC, "call", spy)
    for lv in (0, 2):
        monkeypatch.setattr(OC, "_FUSED_PW_BWD", lv)
        initializers.set_seed(5)
        blocks = [R.Bottleneck(128, stride=2, project=True), R.Bottleneck(128), R.Bottleneck(128)]
        with torch.no_grad():
            h = x
            for b in blocks:
                h = b(h, training=False)
        params = [w for b in blocks for w in b.trainable_weights]
        arena = ParamArena(params, device=cuda)
        seen.clear()
        xx = x.clone().requires_grad_(True)
        h = xx
        for b in blocks:
            h = b(h, training=True)
        loss = (h.float() * torch.linspace(-1, 1, h.shape[-1], device=cuda)).square().mean()
        with direct_grads():
            loss.backward()
        torch.cuda.synchronize()
        runs[lv] = [xx.grad.float(), arena.grad.clone()]
        assert seen.get("dtf_pw_conv_bwd_bn", 0) == (1 if lv else 0), seen
    for a, b in zip(runs[0], runs[2]):
        assert torch.isfinite(b).all()
        err = (a - b).norm().item() / (a.norm().item() + 1e-12)
        assert err < 1e-2, err


def test_pw_bwd_bn_shortcut_partials(cuda):
    """The projection-shortcut BN-backward reduction taken inside the BN-folded pass equals the one the standalone
    apply pass takes (bn_bwd_apply_kernel<true>): sum dz and sum dz (ysc - mean) per channel."""
    P, K, C = 65536 + 37, 256, 64
    g = torch.Generator(device="cpu").manual_seed(23)
    dout = torch.randn(P, K, generator=g).to(BF).to(cuda)
    y = torch.randn(P, K, generator=g).to(BF).to(cuda)
    ysc = torch.randn(P, K, generator=g).to(BF).to(cuda)
    msc = (torch.randn(K, generator=g) * 0.1).to(cuda)
    ym = _bits(torch.rand(P, K, generator=g) > 0.3).to(cuda)
    coef = torch.cat([torch.rand(K, generator=g) + 0.5, torch.randn(K, generator=g) * 0.1,
                      torch.randn(K, generator=g) * 0.01]).to(cuda)
    x = torch.relu(torch.randn(P, C, generator=g)).to(BF).to(cuda)
    wck = (torch.randn(C, K, generator=g) * K ** -0.5).to(BF).to(cuda)
    ws = torch.empty(32 << 20, dtype=F32, device=cuda)
    dx = torch.empty(P, C, dtype=BF, device=cuda)
    dw = torch.zeros(K, C, device=cuda)
    psc = torch.full((256 * 2 * K,), float("nan"), device=cuda)
    rsc = ctypes.c_int(0)
    call("dtf_pw_conv_bwd_bn", ptr(dout), ptr(y), ptr(ym), ptr(coef), ptr(x), ptr(wck), ptr(dx), ptr(dw), 1,
         None, None, None, None, None, ptr(ws), ws.numel(), P, K, C, ptr(ysc), ptr(msc), ptr(psc),
         ctypes.addressof(rsc), None, stream())
    dyc = torch.empty(P, K, dtype=BF, device=cuda)
    dz = torch.empty(P, K, dtype=BF, device=cuda)
    part2 = torch.empty(4096 * 2 * K, device=cuda)
    rows2 = ctypes.c_int(0)
    call("dtf_bn_bwd_apply_coef", ptr(dout), ptr(ym), ptr(y), P, K, ptr(dyc), ptr(dz), ptr(coef), ptr(ysc), ptr(msc),
         ptr(part2), ctypes.addressof(rows2), stream())
    torch.cuda.synchronize()
    assert rsc.value == 256 and rows2.value > 0
    s1 = psc.view(256, 2 * K).sum(0)
    s2 = part2[: rows2.value * 2 * K].view(rows2.value, 2 * K).sum(0)
    ref = torch.cat([dz.float().sum(0), (dz.float() * (ysc.float() - msc)).sum(0)])
    sc = ref.abs().max().item() + 1.0
    assert torch.allclose(s1, s2, atol=1e-4 * sc, rtol=1e-4)
    assert torch.allclose(s1, ref, atol=1e-3 * sc, rtol=1e-3)


def test_pw_dgrad_recomputes_bn_input(cuda):
    """pwconv.hip MODE 3 with the BN input recomputed per tile (RX: bf16(rx rw^T), the stage-1 c3 output the forward
    did not store) equals MODE 3 reading the materialised BN input: dX and the partial rows bitwise (same values,
    same order); plain and compact-shortcut forms."""
    from distributed_tensorflow_amd.ops._util import bf16_shadow
    for imgs, H, W, Kc, sub2 in ((16, 32, 32, 64, False), (16, 32, 32, 128, True)):
        M, N = imgs * H * W, 256
        g = torch.Generator(device="cpu").manual_seed(Kc)
        dy = torch.randn(M, Kc, generator=g).to(BF).to(cuda)
        wck = (torch.randn(N, Kc, generator=g) * Kc ** -0.5).to(BF).to(cuda)
        rx = torch.relu(torch.randn(M, 64, generator=g)).to(BF).to(cuda)
        rw = (torch.randn(N, 64, generator=g) * 0.125).to(BF).to(cuda)
        y = OC._recompute_y(rx, rw, (imgs, H, W, 64, N))
        ref_y = (rx.float() @ rw.float().t()).to(BF)
        assert (y.view(M, N).float() - ref_y.float()).abs().max().item() <= 1e-2 * ref_y.float().abs().max().item()
        mask = _bits(torch.rand(M, N, generator=g) > 0.5).to(cuda)
        mean = (torch.randn(N, generator=g) * 0.1).to(cuda)
        s2 = torch.randn(imgs, H // 2, W // 2, N, generator=g).to(BF).to(cuda) if sub2 else None
        acc = None if sub2 else torch.randn(M, N, generator=g).to(BF).to(cuda)
        outs = []
        for mode in ("stored", "rx"):
            dx = acc.clone() if acc is not None else torch.empty(M, N, dtype=BF, device=cuda)
            part = torch.full(((M + 63) // 64 * 2 * N,), float("nan"), device=cuda)
            rows = ctypes.c_int(0)
            ws = torch.empty(16, dtype=BF, device=cuda)
            bnx = y if mode == "stored" else None
            rr = (ptr(rx), ptr(rw)) if mode == "rx" else (None, None)
            call("dtf_conv_dgrad_x", ptr(dy), ptr(wck), ptr(dx), imgs, H, W, N, Kc, 1, 1, H, W, 1, 1, 0, 0, 1, 1,
                 1.0 if acc is not None else 0.0, ptr(ws), 16, ptr(bnx), ptr(mask), ptr(mean), ptr(part),
                 ctypes.addressof(rows), None, ptr(s2), *rr, stream())
            torch.cuda.synchronize()
            outs.append((dx, part[: rows.value * 2 * N].clone(), rows.value))
        (a, pa, ra), (b, pb, rb) = outs
        assert ra == rb and ra <= 256
        assert torch.equal(a.view(torch.int16), b.view(torch.int16))
        assert torch.equal(pa, pb)


def test_unstored_y_falls_back_when_the_consumer_cannot_recompute(cuda, monkeypatch):
    """Level 4 with the persistent pointwise data gradient switched off: the next block's c1 data gradient cannot
    recompute the unstored c3 output (dtf_conv_dgrad_x returns -12, nothing launched), so it is materialised once
    (_BNSource.materialize) — gradients equal the level-0 path's to f32 summation order."""
    from distributed_tensorflow_amd.keras import initializers
    from distributed_tensorflow_amd.models import resnet as R
    from distributed_tensorflow_amd.ops._util import direct_grads
    from distributed_tensorflow_amd.variables import ParamArena
    g = torch.Generator().manual_seed(29)
    x = torch.randn(64, 16, 16, 64, generator=g).to(cuda).to(BF)
    runs = {}
    mats = []
    real = OC._recompute_y

    def spy(*a):
        mats.append(1)
        return real(*a)

    monkeypatch.setattr(OC, "_recompute_y", spy)
    call("dtf_set_pw_dgrad", 0)
    try:
        for lv in (0, 4):
            monkeypatch.setattr(OC, "_FUSED_PW_BWD", lv)
            mats.clear()
            initializers.set_seed(3)
            blocks = [R.Bottleneck(64, stride=1, project=True), R.Bottleneck(64), R.Bottleneck(64)]
            with torch.no_grad():
                h = x
                for b in blocks:
                    h = b(h, training=False)
            params = [w for b in blocks for w in b.trainable_weights]
            arena = ParamArena(params, device=cuda)
            xx = x.clone().requires_grad_(True)
            h = xx
            for b in blocks:
                h = b(h, training=True)
            loss = (h.float() * torch.linspace(-1, 1, h.shape[-1], device=cuda)).square().mean()
            with direct_grads():
                loss.backward()
            torch.cuda.synchronize()
            runs[lv] = [xx.grad.float(), arena.grad.clone()]
            if lv == 4:
                assert len(mats) >= 2, mats  # b1 / b2 c1 dgrads materialised the unstored BN inputs
    finally:
        call("dtf_set_pw_dgrad", 1)
    for a, b in zip(runs[0], runs[4]):
        assert torch.isfinite(b).all()
        err = (a - b).norm().item() / (a.norm().item() + 1e-12)
        assert err < 1e-2, err
