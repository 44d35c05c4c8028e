"""NHWC Conv2D (+ fused FusedBatchNorm / residual / ReLU) on the gfx950 implicit-GEMM kernel.

Activations are channels-last ``[N, H, W, C]`` bf16; filters are stored KRSC
(``[out, kh, kw, in]``) as f32 master variables with a bf16 compute shadow.
The training-mode BatchNorm statistics are produced by the conv epilogue
(per-M-tile partial sum / sum^2 rows, reduced deterministically by bn_finalize)
so the forward BN costs one apply pass
instead of three (SURVEY §2.4.b K4/K5, §7.4 hard part 1).
"""
from __future__ import annotations

import os

import torch

from ._util import (BF16, F32, SIDE_STREAM_ON, IntOut, K as K_, before_overwrite, bf16_shadow, call, crsk_shadow,
                    direct_grad, fork_side, mark_parked, on_gpu, ptr, stream, workspace)


def out_size(h, k, s, p, d=1):
    return (h + 2 * p - d * (k - 1) - 1) // s + 1


def same_pads(h, k, s, d=1):
    """TF 'SAME' padding (pad_top, pad_total) for one spatial dim."""
    out = (h + s - 1) // s
    total = max((out - 1) * s + (k - 1) * d + 1 - h, 0)
    return total // 2, total


def _geom(x, w, stride, pad, dil):
    N, H, W, C = x.shape
    K, R, S, C2 = w.shape
    assert C == C2, f"channel mismatch {C} vs {C2}"
    sh, sw = stride
    ph, pw = pad
    dh, dw = dil
    P = out_size(H, R, sh, ph, dh)
    Q = out_size(W, S, sw, pw, dw)
    return N, H, W, C, K, R, S, P, Q, sh, sw, ph, pw, dh, dw


def conv_fwd_raw(x, w16, g, stats=False, bias=None, act=0):
    """Returns y, or (y, partials, rows) when stats: BN partial sums, one [2K] row per M-tile."""
    N, H, W, C, K, R, S, P, Q, sh, sw, ph, pw, dh, dw = g
    y = torch.empty((N, P, Q, K), dtype=BF16, device=x.device)
    part = rows = None
    if stats:
        part = torch.empty(((N * P * Q + 63) // 64) * 2 * K, dtype=F32, device=x.device)
        rows = IntOut()
    call("dtf_conv_fwd", ptr(x), ptr(w16), ptr(y), ptr(bias), ptr(part), rows.addr if rows else None, N, H, W, C,
         K, R, S, P, Q, sh, sw, ph, pw, dh, dw, int(act), 0, -1, stream())
    if stats:
        return y, part, rows.value
    return y


def conv_fwd_bn_raw(x, w16, g, gamma, beta, rmean, rvar, momentum, eps, scale, shift, mean, invstd):
    """Training ConvBN forward: y plus the output BatchNorm's scale/shift/mean/invstd and running-statistics update,
    finalized inside the conv launch's tail (gemm_core.h BnFin) — or by the separate reduction + finalize launches
    when the launch cannot (the native side falls back by itself)."""
    N, H, W, C, K, R, S, P, Q, sh, sw, ph, pw, dh, dw = g
    y = torch.empty((N, P, Q, K), dtype=BF16, device=x.device)
    part = torch.empty(((N * P * Q + 63) // 64) * 2 * K, dtype=F32, device=x.device)
    call("dtf_conv_fwd_bn", ptr(x), ptr(w16), ptr(y), ptr(part), N, H, W, C, K, R, S, P, Q, sh, sw, ph, pw, dh, dw,
         -1, ptr(gamma), ptr(beta), ptr(rmean), ptr(rvar), float(momentum), float(eps), ptr(scale), ptr(shift),
         ptr(mean), ptr(invstd), None, stream())
    return y


def conv_dgrad_raw(dy, w_master, g, acc=None, bn=None, acc_mask=None, acc_sub2=None):
    """dX (bf16); with `acc` (a bf16 [N,H,W,C] gradient already holding another contribution) the epilogue
    adds into it (beta = 1) and returns it; `acc_mask` (1 bit per element) first zeroes the acc values whose
    bit is clear (a residual gradient whose ReLU mask was deferred). With `bn` (the _BNSource of the
    BatchNorm whose output this conv consumed) the epilogue also produces that BatchNorm's backward
    reduction of the final dX values and stores it on `bn` (see _BNSource)."""
    N, H, W, C, K, R, S, P, Q, sh, sw, ph, pw, dh, dw = g
    wc = crsk_shadow(w_master, K, R * S, C)
    dx = torch.empty((N, H, W, C), dtype=BF16, device=dy.device) if acc is None else acc
    ws = workspace(dy.device)  # strided convs: per-phase compact filters (bf16) live here
    part = rows = None
    if bn is not None:
        # one partial row per M-tile (>= 64 rows) of every launch: a strided dgrad runs sh*sw phase launches,
        # each of which may end in a partial tile
        part = torch.empty(((N * H * W + 63) // 64 + sh * sw) * 2 * C, dtype=F32, device=dy.device)
        rows = IntOut()
    bn_ptrs = ((ptr(bn.yc), ptr(bn.mbits), ptr(bn.mean)) if bn is not None else (None, None, None))
    if acc_sub2 is not None:  # + the compact gradient of a stride-2 1x1 shortcut at the even pixels
        assert acc is None and (R, S, sh, sw, ph, pw) == (1, 1, 1, 1, 0, 0)
    rx = (ptr(bn.rx), ptr(bf16_shadow(bn.rw))) if (bn is not None and bn.yc is None) else (None, None)
    args = (ptr(dy), ptr(wc), ptr(dx), N, H, W, C, K, R, S, P, Q, sh, sw, ph, pw, dh, dw,
            1.0 if (acc is not None or acc_sub2 is not None) else 0.0, ptr(ws), 2 * ws.numel())
    tail = (ptr(part), rows.addr if rows else None, ptr(acc_mask) if acc is not None else None, ptr(acc_sub2))
    rc = K_().dtf_conv_dgrad_x(*args, None, ptr(bn.mbits), ptr(bn.mean), *tail, *rx, stream()) if rx[0] else -12
    if rc == -12:  # (the BN input is stored, or only the persistent pointwise route can recompute it)
        if bn is not None:
            bn_ptrs = (ptr(bn.materialize()), ptr(bn.mbits), ptr(bn.mean))
        call("dtf_conv_dgrad_x", *args, *bn_ptrs, *tail, None, None, stream())
    elif rc != 0:
        raise RuntimeError(f"dtf_conv_dgrad_x failed with status {rc}")
    if bn is not None:
        bn.provide(dx, part, rows.value)
    return dx


def _recompute_y(x, w, g):
    """bf16(x w^T) of a stage-1 channel-expanding 1x1 conv whose output was not stored, with the pointwise forward
    kernel the two-pass forward used (the same MFMA sequence: bitwise its values)."""
    N, H, W, C, K = g[:5]
    M = N * H * W
    y = torch.empty((N, H, W, K), dtype=BF16, device=x.device)
    stats = torch.empty(((M + 63) // 64) * 2 * K, dtype=F32, device=x.device)
    rows = IntOut()
    call("dtf_pwconv_fwd", ptr(x), ptr(bf16_shadow(w)), ptr(y), ptr(stats), rows.addr, M, C, K, stream())
    return y


def pw_bwd_ok(g, M_min=64 * 256):
    """Shapes of the fused 1x1 data + weight gradient (pwbwd.hip): stride-1 unpadded 1x1, K_out 256 from C_in 64
    (ResNet-50 stage-1 c3 and stride-1 projection), >= 256 pixel tiles, tensors < 2 GiB."""
    N, H, W, C, K, R, S, P, Q, sh, sw, ph, pw = g[:13]
    M = N * P * Q
    return ((R, S, sh, sw, ph, pw) == (1, 1, 1, 1, 0, 0) and K == 256 and C == 64 and M >= M_min
            and M * K * 2 < (1 << 31))


def pw_bwd_bn_ok(g):
    """Shapes of the BatchNorm-folded form (dtf_pw_conv_bwd_bn): stage 1 (K_out 256 from 64, >= 256 64-pixel tiles)
    or stage 2 (K_out 512 from 128, >= 128 32-pixel tiles)."""
    N, H, W, C, K, R, S, P, Q, sh, sw, ph, pw = g[:13]
    M = N * P * Q
    if (R, S, sh, sw, ph, pw) != (1, 1, 1, 1, 0, 0) or M * K * 2 >= (1 << 31):
        return False
    return (K, C) == (256, 64) and M >= 64 * 256 or (K, C) == (512, 128) and M >= 32 * 128


def conv_bwd_fused_raw(dy, x, w_master, g, dw_out, bn=None):
    """dX (bf16) and dW += (into the f32 arena gradient dw_out) of a pw_bwd_ok conv in ONE pass over dy
    (pwbwd.hip); with `bn` (the _BNSource of the BatchNorm that produced x, see conv_dgrad_raw) the BN-backward
    partial rows of dX go to it."""
    N, H, W, C, K = g[:5]
    M = N * H * W
    wc = crsk_shadow(w_master, K, 1, C)
    dx = torch.empty((N, H, W, C), dtype=BF16, device=dy.device)
    ws = workspace(dy.device)
    part = rows = None
    if bn is not None:
        part = torch.empty(256 * 2 * C, dtype=F32, device=dy.device)
        rows = IntOut()
    bn_ptrs = ((ptr(bn.materialize()), ptr(bn.mbits), ptr(bn.mean)) if bn is not None else (None, None, None))
    call("dtf_pw_conv_bwd", ptr(dy), ptr(x), ptr(wc), ptr(dx), ptr(dw_out), 1, *bn_ptrs, ptr(part),
         rows.addr if rows else None, ptr(ws), ws.numel(), M, K, C, stream())
    if bn is not None:
        bn.provide(dx, part, rows.value)
    return dx


def conv_bwd_bn_fused_raw(dout, y, ymask, coef, x, w_master, g, dw_out, bn=None, sc=None, wy=None):
    """conv_bwd_fused_raw with dy = a*dz + b*y + c (the BatchNorm(+ReLU) backward of y = conv output, coefficients
    coef [3K] from dtf_bn_bwd_coef, dz = dout under the ReLU bits ymask) computed inside the kernel. With `sc` (the
    _BNSource of a deferred projection-shortcut BN added as this layer's residual) the kernel also takes that BN's
    backward reduction of dz and provides it to the source for `dout`. With `wy` (the layer's bf16 forward filter) and
    y None, y is recomputed per tile from x (it was not stored).""" 
    N, H, W, C, K = g[:5]
    M = N * H * W
    wc = crsk_shadow(w_master, K, 1, C)
    dx = torch.empty((N, H, W, C), dtype=BF16, device=dout.device)
    ws = workspace(dout.device)
    part = rows = None
    if bn is not None:
        part = torch.empty(256 * 2 * C, dtype=F32, device=dout.device)  # (<= 256 pixel slots)
        rows = IntOut()
    bn_ptrs = ((ptr(bn.materialize()), ptr(bn.mbits), ptr(bn.mean)) if bn is not None else (None, None, None))
    psc = rsc = None
    if sc is not None:
        psc, rsc = torch.empty(256 * 2 * K, dtype=F32, device=dout.device), IntOut()
    call("dtf_pw_conv_bwd_bn", ptr(dout), ptr(y), ptr(ymask), ptr(coef), ptr(x), ptr(wc), ptr(dx), ptr(dw_out), 1,
         *bn_ptrs, ptr(part), rows.addr if rows else None, ptr(ws), ws.numel(), M, K, C,
         ptr(sc.yc) if sc is not None else None, ptr(sc.mean) if sc is not None else None, ptr(psc),
         rsc.addr if rsc else None, ptr(wy), stream())
    if bn is not None:
        bn.provide(dx, part, rows.value)
    if sc is not None:
        sc.provide(dout, psc, rsc.value)
    return dx


def conv_wgrad_raw(x, dy, g, out=None):
    """dW [K,R,S,C] f32; with `out` (an arena gradient view) the result is accumulated into it."""
    N, H, W, C, K, R, S, P, Q, sh, sw, ph, pw, dh, dw = g
    dw_ = torch.empty((K, R, S, C), dtype=F32, device=x.device) if out is None else out
    ws = workspace(x.device)
    call("dtf_conv_wgrad", ptr(x), ptr(dy), ptr(dw_), N, H, W, C, K, R, S, P, Q, sh, sw, ph, pw, dh, dw,
         int(out is not None), 0, -1, ptr(ws), ws.numel(), stream())
    return dw_


_STEM_WGRAD = os.environ.get("DTF_STEM_WGRAD", "1") != "0"  # A/B switch: 0 keeps the general wgrad tiles
# 1: the s2d stem's BN + ReLU + MaxPool backward is applied inside the stem wgrad kernel (dtf_stem_wgrad_fused)
_STEM_WGRAD_FUSED = _STEM_WGRAD and os.environ.get("DTF_STEM_WGRAD_FUSED", "1") != "0"


def stem_wgrad_raw(x, dy, g):
    """dW [64, 4, 4, 16] f32 of the space-to-depth stem conv (valid 4x4/1 over the s2d image x [N, Hs, Ws, 16]): the
    persistent stem kernel (csrc/kernels/stemwgrad.hip: the filter gradient resident in the accumulators, one dY row
    image and a ring of s2d rows in LDS, taps as pixel shifts), or the general tiles when it does not take the shape."""
    N, H, W, C, K, R, S, P, Q, sh, sw, ph, pw, dh, dw = g
    if (_STEM_WGRAD and on_gpu(x) and (C, K, R, S, sh, sw, ph, pw, dh, dw) == (16, 64, 4, 4, 1, 1, 0, 0, 1, 1)
            and x.is_contiguous() and dy.is_contiguous()):
        dw_ = torch.empty((K, R, S, C), dtype=F32, device=x.device)
        ws = workspace(x.device)
        if K_().dtf_stem_wgrad(ptr(x), ptr(dy), ptr(dw_), N, H, W, 0, ptr(ws), ws.numel(), stream()) == 0:
            return dw_
    return conv_wgrad_raw(x, dy, g)


class _ConvFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, stride, pad, dil, act):
        x = x.contiguous()
        g = _geom(x, w, stride, pad, dil)
        y = conv_fwd_raw(x, bf16_shadow(w), g, bias=b, act=act)
        ctx.save_for_backward(x, w, y if act else None)
        ctx.g = g
        ctx.act = act
        ctx.has_b = b is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w, y = ctx.saved_tensors
        dy = dy.to(BF16).contiguous()
        if ctx.act == 1:
            dz = torch.empty_like(dy)
            call("dtf_act", ptr(y), ptr(dy), ptr(dz), dz.numel(), 1, 1, stream())  # relu'(y) == relu'(pre)
            dy = dz
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = conv_dgrad_raw(dy, w, ctx.g)
        if ctx.needs_input_grad[1]:
            dw = conv_wgrad_raw(x, dy, ctx.g)
        if ctx.has_b and ctx.needs_input_grad[2]:
            db = torch.empty(dy.shape[-1], dtype=F32, device=dy.device)
            call("dtf_colsum", ptr(dy), dy.numel() // dy.shape[-1], dy.shape[-1], ptr(db), 0, stream())
        return dx, dw, db, None, None, None, None


def _ref_conv(x, w, b, stride, pad, dil):
    y = torch.nn.functional.conv2d(x.permute(0, 3, 1, 2).to(w.dtype), w.permute(0, 3, 1, 2), b, stride=stride,
                                   padding=pad, dilation=dil)
    return y.permute(0, 2, 3, 1)


def conv2d(x, w, b=None, stride=(1, 1), pad=(0, 0), dil=(1, 1), act=0):
    """NHWC conv; w is KRSC. Explicit symmetric padding (use same_pads for TF SAME)."""
    stride, pad, dil = tuple(stride), tuple(pad), tuple(dil)
    if on_gpu(x):
        return _ConvFn.apply(x.to(BF16), w, b, stride, pad, dil, act)
    y = _ref_conv(x, w, b, stride, pad, dil)
    return torch.relu(y) if act == 1 else y


class ResidualGradLink:
    """Joins the two gradient contributions of a residual block's input without an extra add pass.

    The block input x feeds the first conv (role "acc") and the shortcut: either directly as the residual of
    the last conv (role "res") or through a projection conv (role "proj"). The shortcut's backward parks its
    gradient of x here instead of returning it, and the first conv's dgrad epilogue adds into that buffer
    (beta = 1) and returns the sum — autograd sees one gradient for x and runs no add kernel. If the first
    conv's backward happens to run before the projection's (autograd schedules by creation order; the block
    creates the projection after the first conv so that it runs first), the link closes and both return their
    gradients normally, so the result is the same either way.

    An identity shortcut may park LAZILY: the last conv's BatchNorm(+ReLU) backward then parks its incoming
    gradient together with the ReLU mask instead of writing the masked residual gradient, and the first conv's
    epilogue applies the mask while adding (one activation-sized write saved per identity block; the parked
    tensor is overwritten in place, it has no other reader).

    A stride-2 1x1 projection may park its data gradient COMPACT ([N, H/2, W/2, C], the only pixels it reaches):
    the first conv's dgrad epilogue then adds it at the even pixels of its own full-size output, so the
    projection's full-size gradient (3/4 zeros) is never cleared, written or read.
    """
    __slots__ = ("buf", "mask", "closed", "compact")

    def __init__(self):
        self.buf = None
        self.mask = None
        self.closed = False
        self.compact = False

    def park(self, g, mask=None, compact=False):
        """Shortcut side: returns what to hand autograd (None when parked)."""
        if self.closed or g is None:
            assert not compact, "a compact gradient can only be parked on an open link"
            return g
        self.buf, self.mask, self.compact = g, mask, compact
        mark_parked(g)
        return None

    def take(self):
        """First-conv side: (parked gradient to accumulate into, its deferred ReLU mask or None, compact flag), or
        (None, None, False); then the link closes."""
        buf, mask, compact = self.buf, self.mask, self.compact
        self.buf = self.mask = None
        self.compact = False
        if buf is None:
            self.closed = True
        else:
            before_overwrite(buf)  # side-stream readers of the parked gradient finish first
        return buf, mask, compact


class _BNSource:
    """What the consumer of a training-mode ConvBN output needs to fuse that BatchNorm's backward reduction
    into its own data-gradient GEMM: the BN input (conv output) yc, the 1-bit ReLU mask and the batch mean.

    Attached to the ConvBN output tensor. A consuming ConvBN whose dgrad produces the COMPLETE gradient of
    that output (its only consumer, or the residual-link "acc" conv that also adds the shortcut's parked
    gradient) lets the GEMM epilogue write sum(dz), sum(dz*(x-mean)) partial rows; the producing ConvBN's
    backward then skips its reduction pass (bn_bwd_reduce), provided the gradient it receives is exactly the
    tensor that dgrad wrote (same storage: autograd added nothing else to it)."""
    __slots__ = ("yc", "mbits", "mean", "invstd", "gamma", "gamma_p", "beta_p", "consumers", "part", "rows", "dx",
                 "ver", "rx", "rw", "g", "__weakref__")

    def __init__(self, yc, mbits, mean, invstd=None, gamma=None, params=(None, None), recompute=None):
        self.yc, self.mbits, self.mean = yc, mbits, mean
        self.invstd, self.gamma = invstd, gamma
        self.gamma_p, self.beta_p = params
        self.consumers = 0
        self.part = self.rows = self.dx = self.ver = None
        # yc not stored: it is bf16(rx rw^T), the producing 1x1 conv's output (input rx, filter parameter rw, geometry
        # g), recomputed by the consumers that can (pwconv.hip RX, pwbwd.hip YR) or materialised on demand
        self.rx, self.rw, self.g = recompute if recompute is not None else (None, None, None)

    def materialize(self):
        """The BN input yc, recomputed once (bitwise the forward's values) if it was not stored."""
        if self.yc is None:
            self.yc = _recompute_y(self.rx, self.rw, self.g)
        return self.yc

    def provide(self, dx, part, rows):
        # dx itself is held (not its address), with its version: see nn.same_unmodified
        self.part, self.rows, self.dx, self.ver = part, rows, dx, dx._version

    def take(self, dout):
        """("partials", part, rows) for this gradient, or None (then the regular reduction runs)."""
        from .nn import same_unmodified
        part, rows, dx, ver = self.part, self.rows, self.dx, self.ver
        self.part = self.rows = self.dx = self.ver = None
        if not same_unmodified(dout, dx, ver):
            return None
        if part is None or rows < 1:
            return None
        return "partials", part, rows


# Fused BatchNorm backward reduction in the consumer's data-gradient GEMM (see _BNSource), lazy residual gradient
# (parked with its ReLU mask on the link), deferred projection-shortcut BN and the compact stride-2 shortcut
# gradient: module switches for tests (tests/test_resnet_gpu.py flips them to compare against the plain path).
_FUSE_BN_BWD = True
_LAZY_RES = True
_DEFER_PROJ_BN = True
_COMPACT_PROJ = True
# Two-pass forward of the channel-expanding 1x1 ConvBN (statistics pass + recomputed product with the BN apply in its
# epilogue, pwconv.hip dtf_conv_bn_apply_fwd) instead of conv(+stats) -> finalize -> standalone apply pass.
_TWO_PASS_PW = os.environ.get("DTF_PW2", "1") != "0"
# Fused data + weight gradient of the stage-1 channel-reducing 1x1 convs (pwbwd.hip): one read of dY for both,
# the weight gradient on the main stream instead of the side stream.
# Level 2 also folds the conv output's BatchNorm(+ReLU) backward into that pass when its reduction is already done
# (identity blocks: dY = a dz + b y + c computed per tile, never stored: the standalone apply pass disappears).
# Level 3 stops storing the stage-1 identity blocks' c3 output y at all: the folded pass and the next
# block's c1 data gradient recompute it per tile from the c3 input (bitwise the forward's values); level 4 (default) also the
# projection block's.
_FUSED_PW_BWD = int(os.environ.get("DTF_PW_BWD", "4"))


def _two_pass_ok(g):
    """Shapes the two-pass pointwise forward handles (pwconv.hip pw_plan): stride-1 unpadded 1x1, C_in 64/128/256,
    K_out = 256 x {1, 2, 4, 8}, tensors < 2 GiB, >= 8 row tiles."""
    N, H, W, C, K, R, S, P, Q, sh, sw, ph, pw, dh, dw = g
    if (R, S, sh, sw, ph, pw) != (1, 1, 1, 1, 0, 0) or C not in (64, 128, 256) or K % 256 or K // 256 not in (1, 2, 4, 8):
        return False
    M = N * P * Q
    return M * K * 2 < (1 << 31) and M * C * 2 < (1 << 31) and M >= 8 * (128 if C == 64 else 64)
# (Measured and removed: "lazy" BatchNorm outputs applied by the consuming conv's operand loaders, r3 —
# profiles/r3_lazy_bn_modes.txt; the BN finalize inside the producing GEMM launch and a BN apply that recomputes the
# expanding 1x1 product, r4 — profiles/r4_negative_results.txt.)


class _ConvBNFn(torch.autograd.Function):
    """y = [relu]( BN_train(conv(x, w)) [+ residual] ) with batch statistics from the conv epilogue."""

    @staticmethod
    def forward(ctx, x, w, gamma, beta, res, rmean, rvar, stride, pad, dil, relu, momentum, eps, training,
                link=None, role=None):
        in_src = getattr(x, "_dtf_bnsrc", None)
        if in_src is not None:
            in_src.consumers += 1
        if res is not None and getattr(res, "_dtf_bnsrc", None) is not None:
            res._dtf_bnsrc.consumers += 1
        x = x.contiguous()
        g = _geom(x, w, stride, pad, dil)
        N, H, W, C, K, R, S, P, Q = g[:9]
        M = N * P * Q
        dev = x.device
        work = torch.empty(4 * K, dtype=F32, device=dev)  # scale shift mean invstd
        scale, shift, mean, invstd = work[:K], work[K:2 * K], work[2 * K:3 * K], work[3 * K:]
        raff = getattr(res, "_dtf_affine", None) if res is not None else None
        deferred = role == "proj" and not relu and _DEFER_PROJ_BN
        out = mbits = None
        if training and not deferred and _TWO_PASS_PW and _two_pass_ok(g):
            # channel-expanding 1x1 (bottleneck c3): statistics pass, finalize, then the recomputed product with the
            # BatchNorm / residual / ReLU applied in the epilogue (pwconv.hip MODE 1 / 2) — no standalone apply pass
            # level 3: an identity block's stage-1 c3 output is not stored at all — its consumers (this layer's
            # BatchNorm-folded backward, the next block's c1 data gradient) recompute it from x and w
            keep_y = not (_FUSED_PW_BWD >= 3 and (C, K) == (64, 256) and relu and res is not None
                          and M >= 64 * 256 and any(ctx.needs_input_grad)
                          and ((raff is None and link is not None and role == "res")
                               or (_FUSED_PW_BWD >= 4 and raff is not None)))
            yc = torch.empty((N, P, Q, K), dtype=BF16, device=dev) if keep_y else None
            out = torch.empty((N, P, Q, K), dtype=BF16, device=dev)
            mbits = torch.empty(M * K // 8, dtype=torch.uint8, device=dev) if relu else None
            part = torch.empty(((M + 63) // 64) * 2 * K, dtype=F32, device=dev)
            rc_ = res.contiguous() if res is not None else None
            call("dtf_conv_bn_apply_fwd", ptr(x), ptr(bf16_shadow(w)), ptr(yc), ptr(out), ptr(mbits), ptr(rc_),
                 ptr(raff[0]) if raff else None, ptr(raff[1]) if raff else None, M, C, K, int(relu), ptr(part),
                 ptr(gamma), ptr(beta), ptr(rmean), ptr(rvar), float(momentum), float(eps), ptr(scale), ptr(shift),
                 ptr(mean), ptr(invstd), stream())
        elif training:
            yc = conv_fwd_bn_raw(x, bf16_shadow(w), g, gamma, beta, rmean, rvar, momentum, eps, scale, shift, mean,
                                 invstd)
        else:
            yc = conv_fwd_raw(x, bf16_shadow(w), g)
            call("dtf_bn_infer_coeff", ptr(gamma), ptr(beta), ptr(rmean), ptr(rvar), K, float(eps), ptr(scale),
                 ptr(shift), stream())
            if any(ctx.needs_input_grad):  # frozen BN: the backward normalises with the running statistics
                mean.copy_(rmean)
                torch.rsqrt(rvar + eps, out=invstd)
        # the deferred projection BN (its input + mean): its backward reduction is taken in our apply pass
        res_src = getattr(res, "_dtf_bnsrc", None) if raff is not None else None
        if res is not None:
            res = res.contiguous()
        if out is not None:  # (the two-pass form above already wrote out and mbits)
            pass
        elif deferred:
            # projection shortcut: its BN output is consumed only as the residual of the block's last ConvBN,
            # whose apply pass normalises the conv output on the fly (res * scale + shift) — hand autograd the
            # conv output tagged with the affine instead of materialising the BN output
            out = yc
            out._dtf_affine = (scale, shift)
        else:
            mbits = torch.empty(M * K // 8, dtype=torch.uint8, device=dev) if relu else None
            out = torch.empty_like(yc)
            call("dtf_bn_apply", ptr(yc), ptr(scale), ptr(shift), ptr(res), ptr(out), M, K, int(relu), ptr(mbits),
                 ptr(raff[0]) if raff else None, ptr(raff[1]) if raff else None, stream())
        # backward needs the conv output and a 1-bit ReLU mask, not the bf16 BN output
        ctx.save_for_backward(x, w, gamma, yc, mbits, mean, invstd)
        ctx.bn_params = (gamma, beta)
        ctx.g = g
        ctx.relu = relu
        ctx.has_res = res is not None
        ctx.training = training
        ctx.link, ctx.role = link, role
        ctx.in_src = in_src if (ctx.needs_input_grad[0] and _FUSE_BN_BWD) else None
        ctx.res_src = res_src if (training and _FUSE_BN_BWD) else None
        ctx.src = None
        if training and _FUSE_BN_BWD and any(ctx.needs_input_grad):
            src = _BNSource(yc, mbits, mean, invstd, gamma, (gamma, beta),
                            recompute=(x, w, g) if yc is None else None)
            out._dtf_bnsrc = src
            ctx.src = src
        return out

    @staticmethod
    def backward(ctx, dout):
        x, w, gamma, yc, mbits, mean, invstd = ctx.saved_tensors
        g = ctx.g
        K = g[4]
        M = g[0] * g[7] * g[8]
        yshape, dev = (g[0], g[7], g[8], K), x.device
        # a deferred projection BN whose consumer handed over its raw incoming gradient with the ReLU bits to apply
        # (see the projection-block branch below): dz = dout under that mask
        dmask = getattr(dout, "_dtf_mask", None)
        dout = dout.to(BF16).contiguous()
        if dmask is not None:
            assert mbits is None and not ctx.relu
            mbits = dmask
        if not ctx.training:
            return _ConvBNFn._backward_frozen(ctx, dout, x, w, gamma, yc, mbits, mean, invstd)
        dyc = torch.empty(yshape, dtype=BF16, device=dev)
        link, role = ctx.link, ctx.role
        # identity shortcut with ReLU: park dout + the ReLU mask instead of writing the masked residual gradient
        lazy_res = (ctx.has_res and ctx.relu and link is not None and role == "res" and not link.closed
                    and _LAZY_RES and mbits is not None)
        dres = torch.empty(yshape, dtype=BF16, device=dev) if (ctx.has_res and ctx.relu and not lazy_res) else None
        gamma_p, beta_p = ctx.bn_params
        tg, tb = direct_grad(gamma_p), direct_grad(beta_p)
        direct_bn = tg is not None and tb is not None  # accumulate dgamma/dbeta into the arena grads
        dgamma = tg if direct_bn else torch.empty(K, dtype=F32, device=dev)
        dbeta = tb if direct_bn else torch.empty(K, dtype=F32, device=dev)
        fused = ctx.src.take(dout) if ctx.src is not None else None
        rsrc = ctx.res_src if dres is not None else None
        sc = (None, None, None, None)
        if rsrc is not None:  # projection shortcut BN: its backward reduction rides on our apply pass
            part2, rows2 = torch.empty(2048 * 2 * K, dtype=F32, device=dev), IntOut()
            sc = (ptr(rsrc.yc), ptr(rsrc.mean), ptr(part2), rows2.addr)
        if (fused is not None and lazy_res and rsrc is None and _FUSED_PW_BWD >= 2 and ctx.needs_input_grad[0]
                and ctx.needs_input_grad[1] and pw_bwd_bn_ok(g) and x.is_contiguous() and x.dtype == BF16
                and (yc is not None or (g[4], g[3]) == (256, 64))):
            tw = direct_grad(w)
            if tw is not None:
                # identity-block c3: finalize the BN-backward reduction only, then ONE pass computes dY per tile from
                # dout / yc / the ReLU bits and both conv gradients from it (dY is never stored)
                coef = torch.empty(3 * K, dtype=F32, device=dev)
                call("dtf_bn_bwd_coef", ptr(fused[1]), fused[2], ptr(mean), ptr(invstd), ptr(gamma), M, K,
                     ptr(dgamma), ptr(dbeta), int(direct_bn), ptr(coef), stream())
                src = ctx.in_src
                complete = src is not None and src.consumers == 1
                dx = conv_bwd_bn_fused_raw(dout, yc, mbits, coef, x, w, g, tw, bn=src if complete else None,
                                           wy=bf16_shadow(w) if yc is None else None)
                # the identity shortcut's gradient: dout parked with the ReLU mask (read above, in stream order, before
                # the first conv's dgrad overwrites it)
                link.park(dout, mask=mbits)
                ctx.in_src = ctx.src = ctx.res_src = None
                if direct_bn:
                    dgamma = dbeta = None
                return (dx, None, dgamma, dbeta, None, None, None, None, None, None, None, None, None, None, None,
                        None)
        blk_ok = (_FUSED_PW_BWD >= 2 and fused is not None and ctx.needs_input_grad[0] and ctx.needs_input_grad[1]
                  and x.is_contiguous() and x.dtype == BF16)
        if (blk_ok and rsrc is not None and not lazy_res and ctx.relu and pw_bwd_bn_ok(g)
                and g[4] == 256 and g[3] == 64):
            tw = direct_grad(w)
            if tw is not None:
                # projection-block c3 (stage 1): the same one-pass form, also taking the shortcut BN's reduction of
                # dz; the shortcut then receives the raw dout tagged with the ReLU bits instead of a materialised dz
                coef = torch.empty(3 * K, dtype=F32, device=dev)
                call("dtf_bn_bwd_coef", ptr(fused[1]), fused[2], ptr(mean), ptr(invstd), ptr(gamma), M, K,
                     ptr(dgamma), ptr(dbeta), int(direct_bn), ptr(coef), stream())
                src = ctx.in_src
                complete = src is not None and role != "proj" and src.consumers == 1
                dx = conv_bwd_bn_fused_raw(dout, yc, mbits, coef, x, w, g, tw, bn=src if complete else None,
                                           sc=rsrc, wy=bf16_shadow(w) if yc is None else None)
                dout._dtf_mask = mbits
                ctx.in_src = ctx.src = ctx.res_src = None
                if direct_bn:
                    dgamma = dbeta = None
                return (dx, None, dgamma, dbeta, dout, None, None, None, None, None, None, None, None, None, None,
                        None)
        if (blk_ok and yc is not None and dmask is not None and role == "proj" and rsrc is None and pw_bwd_bn_ok(g)
                and g[4] == 256 and g[3] == 64):
            tw = direct_grad(w)
            if tw is not None:
                # the stride-1 projection of that block: its BN backward folded into its own gradient pass
                coef = torch.empty(3 * K, dtype=F32, device=dev)
                call("dtf_bn_bwd_coef", ptr(fused[1]), fused[2], ptr(mean), ptr(invstd), ptr(gamma), M, K,
                     ptr(dgamma), ptr(dbeta), int(direct_bn), ptr(coef), stream())
                dx = conv_bwd_bn_fused_raw(dout, yc, mbits, coef, x, w, g, tw)
                if link is not None:
                    dx = link.park(dx)
                ctx.in_src = ctx.src = ctx.res_src = None
                if direct_bn:
                    dgamma = dbeta = None
                return (dx, None, dgamma, dbeta, None, None, None, None, None, None, None, None, None, None, None,
                        None)
        if yc is None:  # (not stored by the forward and not recomputed inside a fused pass above)
            yc = _recompute_y(x, w, g)
        if fused is not None:  # the consumer's dgrad epilogue already reduced this gradient
            coef = torch.empty(3 * K, dtype=F32, device=dev)
            call("dtf_bn_bwd_partials", ptr(dout), ptr(mbits), ptr(yc), ptr(mean), ptr(invstd), ptr(gamma), M, K,
                 ptr(dyc), ptr(dres), ptr(dgamma), ptr(dbeta), int(direct_bn), ptr(fused[1]), fused[2], ptr(coef),
                 *sc, stream())
        else:
            work = torch.empty((2 * 1024 + 3) * K, dtype=F32, device=dev)
            call("dtf_bn_bwd", ptr(dout), None, ptr(mbits), ptr(yc), ptr(mean), ptr(invstd), ptr(gamma), M, K,
                 ptr(dyc), ptr(dres), ptr(dgamma), ptr(dbeta), int(direct_bn), ptr(work), *sc, stream())
        if rsrc is not None and rows2.value > 0:
            rsrc.provide(dres, part2, rows2.value)
        ctx.res_src = None
        ctx.src = None
        if ctx.has_res and not ctx.relu:
            dres = dout
        if lazy_res:
            dres = link.park(dout, mask=mbits)  # (None: parked; dout is overwritten by the first conv's dgrad)
        elif link is not None and role == "res":
            dres = link.park(dres)
        dx = dw = None
        tw = direct_grad(w) if ctx.needs_input_grad[1] else None
        if (_FUSED_PW_BWD >= 1 and tw is not None and ctx.needs_input_grad[0] and role != "acc" and pw_bwd_ok(g)
                and x.is_contiguous() and x.dtype == BF16):
            src = ctx.in_src
            complete = src is not None and role != "proj" and src.consumers == 1
            dx = conv_bwd_fused_raw(dyc, x, w, g, tw, bn=src if complete else None)
            if link is not None and role == "proj":
                dx = link.park(dx)
            ctx.in_src = None
            if direct_bn:
                dgamma = dbeta = None
            return dx, None, dgamma, dbeta, dres, None, None, None, None, None, None, None, None, None, None, None
        if ctx.needs_input_grad[1]:
            if tw is not None and SIDE_STREAM_ON:
                with fork_side(x.device, x, dyc):  # off the critical path: overlaps the dgrad chain
                    conv_wgrad_raw(x, dyc, g, out=tw)
            else:
                dw = conv_wgrad_raw(x, dyc, g, out=tw)
            if tw is not None:
                dw = None  # (autograd still runs the parameter's AccumulateGrad node with an undefined
                #            gradient, so its post-accumulate hooks — gradient bucketing — fire as usual)
        if ctx.needs_input_grad[0]:
            acc, acc_mask, compact = link.take() if (link is not None and role == "acc") else (None, None, False)
            src = ctx.in_src
            complete = src is not None and role != "proj" and (
                src.consumers == 1 or (role == "acc" and acc is not None and src.consumers == 2))
            N, H, W, C, K, R, S, P, Q, sh, sw, ph, pw = g[:13]
            if (role == "proj" and link is not None and not link.closed and _COMPACT_PROJ
                    and (R, S, sh, sw, ph, pw) == (1, 1, 2, 2, 0, 0) and H == 2 * P and W == 2 * Q):
                # stride-2 1x1 shortcut: its gradient only reaches the even pixels — a plain GEMM over dY rows
                gc = (N, P, Q, C, K, 1, 1, P, Q, 1, 1, 0, 0, 1, 1)
                dx = link.park(conv_dgrad_raw(dyc, w, gc), compact=True)
            elif compact:
                dx = conv_dgrad_raw(dyc, w, g, bn=src if complete else None, acc_sub2=acc)
            else:
                dx = conv_dgrad_raw(dyc, w, g, acc=acc, bn=src if complete else None, acc_mask=acc_mask)
                if link is not None and role == "proj":
                    dx = link.park(dx)
            ctx.in_src = None
        if direct_bn:
            dgamma = dbeta = None
        return dx, dw, dgamma, dbeta, dres, None, None, None, None, None, None, None, None, None, None, None


    @staticmethod
    def _backward_frozen(ctx, dout, x, w, gamma, yc, mbits, mean, invstd):
        """Backward of an inference-mode (frozen) BatchNorm — Keras' BatchNormalization(training=False) under a
        GradientTape, e.g. fine-tuning with frozen statistics: the BN is the fixed affine gamma*invstd*(z - mean) +
        beta of the running statistics, so dz = dy * relu' * gamma*invstd, dgamma = sum(dy relu' xhat),
        dbeta = sum(dy relu'). Rare path: torch ops on the GPU, f32 math."""
        K = yc.shape[-1]
        dz = dout.float()
        if mbits is not None:
            bits = (mbits.view(-1, 1) >> torch.arange(8, device=mbits.device, dtype=torch.uint8)) & 1
            dz = dz * bits.view(dz.shape).to(dz.dtype)
        dzr = dz.reshape(-1, K)
        xhat = (yc.float().reshape(-1, K) - mean) * invstd
        dgamma, dbeta = (dzr * xhat).sum(0), dzr.sum(0)
        gm = gamma if gamma is not None else torch.ones_like(invstd)
        dyc = (dz * (gm * invstd)).to(BF16).contiguous()
        dres = None
        if ctx.has_res:
            dres = dz.to(BF16) if ctx.relu else dout
        dx = dw = None
        if ctx.needs_input_grad[1]:
            dw = conv_wgrad_raw(x, dyc, ctx.g)
        if ctx.needs_input_grad[0]:
            dx = conv_dgrad_raw(dyc, w, ctx.g)
        ctx.in_src = ctx.src = ctx.res_src = None
        return (dx, dw, dgamma if ctx.needs_input_grad[2] else None, dbeta if ctx.needs_input_grad[3] else None,
                dres, None, None, None, None, None, None, None, None, None, None, None)


def conv_bn(x, w, gamma, beta, rmean, rvar, stride=(1, 1), pad=(0, 0), dil=(1, 1), relu=True, residual=None,
            momentum=0.9, eps=1e-5, training=True, link=None, role=None):
    """Fused Conv2D -> FusedBatchNorm -> (+residual) -> ReLU, NHWC. `link`/`role`: see ResidualGradLink."""
    stride, pad, dil = tuple(stride), tuple(pad), tuple(dil)
    if on_gpu(x):
        return _ConvBNFn.apply(x.to(BF16), w, gamma, beta, residual, rmean, rvar, stride, pad, dil, bool(relu),
                               float(momentum), float(eps), bool(training), link, role)
    y = _ref_conv(x, w, None, stride, pad, dil)
    from .norm import batch_norm_ref
    y = batch_norm_ref(y, gamma, beta, rmean, rvar, momentum, eps, training)
    if residual is not None:
        y = y + residual.to(y.dtype)
    return torch.relu(y) if relu else y


class _ConvBNPoolFn(torch.autograd.Function):
    """y = MaxPool( relu( BN_train(conv(x, w)) ) ) — the ResNet stem as one autograd node.

    The BN+ReLU output is never materialised: one pass over the conv output produces the pooled output and an
    argmax byte per pooled element whose bit 7 is the ReLU mask (norm.hip bn_relu_maxpool_fwd_kernel). The
    backward gathers the pooled gradient per conv-output pixel on the fly in the BN backward's reduce and
    apply passes, instead of writing the pool gradient and re-reading it twice."""

    @staticmethod
    def forward(ctx, x, w, gamma, beta, rmean, rvar, stride, pad, dil, momentum, eps, training, pk, ps, pp,
                s2d=False):
        x = x.contiguous()
        w16 = bf16_shadow(w)
        if s2d:  # x: image_to_s2d_bf16 output; w: the 7x7 filter, run as its 4x4 space-to-depth form
            w16 = stem_s2d_filter(w16)
            g = _geom(x, w16, (1, 1), (0, 0), (1, 1))
        else:
            g = _geom(x, w, stride, pad, dil)
        N, H, W, C, K, R, S, P, Q = g[:9]
        M = N * P * Q
        dev = x.device
        work = torch.empty(4 * K, dtype=F32, device=dev)  # scale shift mean invstd
        scale, shift, mean, invstd = work[:K], work[K:2 * K], work[2 * K:3 * K], work[3 * K:]
        if training:
            yc = conv_fwd_bn_raw(x, w16, g, gamma, beta, rmean, rvar, momentum, eps, scale, shift, mean, invstd)
        else:
            yc = conv_fwd_raw(x, w16, g)
            call("dtf_bn_infer_coeff", ptr(gamma), ptr(beta), ptr(rmean), ptr(rvar), K, float(eps), ptr(scale),
                 ptr(shift), stream())
        P2, Q2 = out_size(P, pk[0], ps[0], pp[0]), out_size(Q, pk[1], ps[1], pp[1])
        y = torch.empty((N, P2, Q2, K), dtype=BF16, device=dev)
        arg = torch.empty((N, P2, Q2, K), dtype=torch.uint8, device=dev)
        call("dtf_bn_relu_maxpool_fwd", ptr(yc), ptr(scale), ptr(shift), ptr(y), ptr(arg), N, P, Q, K, P2, Q2,
             pk[0], pk[1], ps[0], ps[1], pp[0], pp[1], stream())
        ctx.save_for_backward(x, w, gamma, yc, arg, mean, invstd)
        ctx.bn_params = (gamma, beta)
        ctx.g = g
        ctx.pool = (P2, Q2, pk, ps, pp)
        ctx.s2d = s2d
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w, gamma, yc, arg, mean, invstd = ctx.saved_tensors
        g = ctx.g
        N, H, W, C, K, R, S, P, Q = g[:9]
        P2, Q2, pk, ps, pp = ctx.pool
        dy = dy.to(BF16).contiguous()
        gamma_p, beta_p = ctx.bn_params
        tg, tb = direct_grad(gamma_p), direct_grad(beta_p)
        direct_bn = tg is not None and tb is not None
        dgamma = tg if direct_bn else torch.empty(K, dtype=F32, device=yc.device)
        dbeta = tb if direct_bn else torch.empty(K, dtype=F32, device=yc.device)
        work = torch.empty((2 * 1024 + 3) * K, dtype=F32, device=yc.device)
        # s2d stem, filter gradient only: the BN + ReLU + pool backward is applied inside the stem wgrad kernel
        # (dtf_stem_wgrad_fused) from the coefficients the reduce pass leaves in work[:3K]; dyc is never formed
        fused = (ctx.s2d and _STEM_WGRAD_FUSED and ctx.needs_input_grad[1] and (K, pk, ps, pp) == (
            64, (3, 3), (2, 2), (1, 1)) and P == 2 * P2 and Q == 2 * Q2 and W <= 128 and C == 16 and R == 4)
        dyc = None if fused else torch.empty_like(yc)
        call("dtf_maxpool_bn_bwd", ptr(dy), ptr(arg), ptr(yc), ptr(mean), ptr(invstd), ptr(gamma), N, P, Q, K, P2,
             Q2, pk[0], pk[1], ps[0], ps[1], pp[0], pp[1], None if fused else ptr(dyc), ptr(dgamma), ptr(dbeta),
             int(direct_bn), ptr(work), stream())
        dx = dw = None
        if fused:
            dw2 = torch.empty((K, R, S, C), dtype=F32, device=x.device)
            ws = workspace(x.device)
            call("dtf_stem_wgrad_fused", ptr(x), ptr(yc), ptr(dy), ptr(arg), ptr(work), ptr(dw2), N, H, W, 0, ptr(ws),
                 ws.numel(), stream())
            dw = stem_s2d_filter_grad(dw2, w.shape)
            tw = direct_grad(w)
            if tw is not None:
                tw.add_(dw)
                dw = None
            if direct_bn:
                dgamma = dbeta = None
            return None, dw, dgamma, dbeta, None, None, None, None, None, None, None, None, None, None, None, None
        if ctx.needs_input_grad[0]:
            if ctx.s2d:
                raise NotImplementedError("no input gradient through the space-to-depth stem (image input)")
            dx = conv_dgrad_raw(dyc, w, g)
        if ctx.needs_input_grad[1]:
            tw = direct_grad(w)
            if ctx.s2d:
                dw = stem_s2d_filter_grad(stem_wgrad_raw(x, dyc, g), w.shape)
                if tw is not None:
                    tw.add_(dw)
            else:
                dw = conv_wgrad_raw(x, dyc, g, out=tw)
            if tw is not None:
                dw = None
        if direct_bn:
            dgamma = dbeta = None
        return dx, dw, dgamma, dbeta, None, None, None, None, None, None, None, None, None, None, None, None


_S2D_IDX = {}


def _s2d_index(Cp, device):
    """Column maps between a 7x7 stem filter [K, 7, 7, Cp] (flattened per output channel, plus one trailing
    zero column) and its space-to-depth form [K, 4, 4, 16]: s2d tap (a, b), channel (dh*2 + dw)*4 + c holds
    filter tap (2a + dh - 1, 2b + dw - 1), channel c (zero outside the 7x7 window or for c >= Cp)."""
    key = (Cp, str(device))
    if key not in _S2D_IDX:
        zero = 49 * Cp
        fwd = torch.full((4 * 4 * 16,), zero, dtype=torch.long)
        back = torch.full((49 * Cp,), 4 * 4 * 16, dtype=torch.long)
        for a in range(4):
            for b in range(4):
                for k in range(16):
                    dh, dw, c = k >> 3, (k >> 2) & 1, k & 3
                    kh, kw = 2 * a + dh - 1, 2 * b + dw - 1
                    if 0 <= kh < 7 and 0 <= kw < 7 and c < Cp:
                        fwd[(a * 4 + b) * 16 + k] = (kh * 7 + kw) * Cp + c
                        back[(kh * 7 + kw) * Cp + c] = (a * 4 + b) * 16 + k
        _S2D_IDX[key] = (fwd.to(device), back.to(device))
    return _S2D_IDX[key]


def _gather_cols(m, idx, ncols):
    """out[:, j] = m[:, idx[j]] of a row-major 2-D matrix, 0 where idx[j] == m.shape[1] (sort.hip dtf_gather_cols on
    the GPU: one launch, no zero-column concatenation)."""
    rows, cols = m.shape
    if on_gpu(m) and m.element_size() in (2, 4):
        m = m.contiguous()
        out = torch.empty((rows, ncols), dtype=m.dtype, device=m.device)
        call("dtf_gather_cols", ptr(m), m.element_size(), rows, cols, ptr(idx), ncols, ptr(out), stream())
        return out
    return torch.cat([m, m.new_zeros(rows, 1)], 1).index_select(1, idx)


class _S2DFilterFn(torch.autograd.Function):
    """stem_s2d_filter as an autograd node (the native column gather has no autograd of its own): the backward is the
    inverse gather stem_s2d_filter_grad. Used where the s2d filter feeds an autograd conv (the frozen-BN stem path)."""

    @staticmethod
    def forward(ctx, w):
        ctx.shape = tuple(w.shape)
        return _s2d_filter_raw(w)

    @staticmethod
    def backward(ctx, g):
        return stem_s2d_filter_grad(g.contiguous(), ctx.shape)


def _s2d_filter_raw(w):
    K, R, S, Cp = w.shape
    assert (R, S) == (7, 7)
    fwd, _ = _s2d_index(Cp, w.device)
    return _gather_cols(w.reshape(K, -1), fwd, fwd.numel()).reshape(K, 4, 4, 16)


def stem_s2d_filter(w):
    """[K, 7, 7, Cp] -> [K, 4, 4, 16]: the 7x7/2 pad-3 filter as a 4x4/1 filter over image_to_s2d_bf16 output
    (differentiable: gradients flow back to the 7x7 filter)."""
    if torch.is_grad_enabled() and w.requires_grad:
        return _S2DFilterFn.apply(w)
    return _s2d_filter_raw(w)


def stem_s2d_filter_grad(dw2, shape):
    """Gradient of stem_s2d_filter: [K, 4, 4, 16] -> [K, 7, 7, Cp] (every filter entry appears once; the padded
    colour channels c >= 4 get zero)."""
    K, R, S, Cp = shape
    _, back = _s2d_index(Cp, dw2.device)
    return _gather_cols(dw2.reshape(K, -1), back, back.numel()).reshape(K, R, S, Cp)


def image_to_s2d_bf16(x_nchw):
    """f32 NCHW images (<= 4 channels, even H, W) -> bf16 2x2 space-to-depth [N, H/2+3, W/2+3, 16] (zero padding
    baked in) for the space-to-depth stem (conv_bn_maxpool(..., s2d=True))."""
    N, C, H, W = x_nchw.shape
    if on_gpu(x_nchw):
        y = torch.empty((N, H // 2 + 3, W // 2 + 3, 16), dtype=BF16, device=x_nchw.device)
        call("dtf_nchw_to_s2d", ptr(x_nchw.float().contiguous()), ptr(y), N, C, H, W, stream())
        return y
    xp = torch.zeros((N, 4, H + 6, W + 6), dtype=x_nchw.dtype)
    xp[:, :C, 4:H + 4, 4:W + 4] = x_nchw
    # [N, 4, Hs, 2, Ws, 2] -> [N, Hs, Ws, dh, dw, c]
    t = xp.reshape(N, 4, (H + 6) // 2, 2, (W + 6) // 2, 2).permute(0, 2, 4, 3, 5, 1)
    return t.reshape(N, (H + 6) // 2, (W + 6) // 2, 16)


def conv_bn_maxpool(x, w, gamma, beta, rmean, rvar, stride=(1, 1), pad=(0, 0), dil=(1, 1), momentum=0.9, eps=1e-5,
                    training=True, pool_size=(3, 3), pool_strides=(2, 2), pool_pad=(1, 1), s2d=False):
    """MaxPool(ReLU(FusedBatchNorm(Conv2D(x)))), NHWC — the ResNet stem fused (see _ConvBNPoolFn).
    s2d=True: x is image_to_s2d_bf16(images) and w the [K, 7, 7, Cp] filter of a 7x7/2 pad-3 conv (run as the
    equivalent 4x4/1 conv over the space-to-depth image: 256 instead of 392 MACs per output, no padded taps)."""
    stride, pad, dil = tuple(stride), tuple(pad), tuple(dil)
    pk, ps, pp = tuple(pool_size), tuple(pool_strides), tuple(pool_pad)
    if s2d:
        assert tuple(w.shape[1:3]) == (7, 7) and stride == (2, 2) and pad == (3, 3) and dil == (1, 1)
    frozen_grad = not training and torch.is_grad_enabled() and any(
        getattr(t, "requires_grad", False) for t in (x, w, gamma, beta))
    if on_gpu(x) and w.shape[0] % 8 == 0 and pk[0] * pk[1] <= 127 and not frozen_grad:
        # (inference-mode BN under a tape takes the unfused pair below: conv_bn's frozen-BN backward + max_pool2d)
        return _ConvBNPoolFn.apply(x.to(BF16), w, gamma, beta, rmean, rvar, stride, pad, dil, float(momentum),
                                   float(eps), bool(training), pk, ps, pp, bool(s2d))
    if s2d:
        w = stem_s2d_filter(w)
        stride, pad = (1, 1), (0, 0)
    from .nn import max_pool2d
    y = conv_bn(x, w, gamma, beta, rmean, rvar, stride, pad, dil, relu=True, momentum=momentum, eps=eps,
                training=training)
    return max_pool2d(y, pk, ps, pp)


def image_to_nhwc_bf16(x_nchw, cpad=8):
    """Device-side input pipeline step: f32 NCHW images -> bf16 NHWC, channels padded to `cpad`."""
    N, C, H, W = x_nchw.shape
    if on_gpu(x_nchw):
        y = torch.empty((N, H, W, cpad), dtype=BF16, device=x_nchw.device)
        call("dtf_nchw_to_nhwc_pad", ptr(x_nchw.contiguous()), ptr(y), N, C, H * W, cpad, stream())
        return y
    y = torch.zeros((N, H, W, cpad), dtype=x_nchw.dtype)
    y[..., :C] = x_nchw.permute(0, 2, 3, 1)
    return y
