"""FP8 (OCP e4m3 / e5m2) projections for GPT-2-medium (csrc/kernels/gemm_fp8.hip).

Every GEMM of an fp8 Dense layer runs on the gfx950 block-scaled MFMA
(``v_mfma_scale_f32_16x16x128_f8f6f4``, unit block scales + per-tensor scales folded into the epilogue,
f32 accumulate) — forward AND backward:

* forward  ``y = x W^T``:  x e4m3 (delayed scaling: the quantize pass of step t records amax(|x|), which sets
  the scale of step t+1), W e4m3 (exact per-tensor scale, requantized once per optimizer step); dequant, bias
  and GELU fused in the epilogue. The same quantize pass writes x^T in fp8 for the weight gradient, so the
  layer saves 1 byte per activation instead of 2.
* backward ``dX = dZ W`` and ``dW += dZ^T X``:  the incoming gradient is quantized to e5m2 (the wider-range
  format; delayed scaling with its own amax) by ONE transposing pass that also folds in the GELU derivative
  and produces the bias-gradient column sums, so the bf16 dZ is never written. dX runs e5m2 x e4m3 (W^T is kept
  in fp8 next to W), dW runs e5m2 x e4m3 over the tokens with split-K f32 slabs accumulated straight into the
  f32 gradient arena.

Master weights, optimizer and the gradient arena stay f32 (the "fp8 compute / high-precision state" recipe).
DTF_FP8_BWD=0 keeps the backward in bf16 against the bf16 weight copies (forward-only fp8).
"""
from __future__ import annotations

import os

import torch

import contextlib

from ._util import BF16, F32, K, bf16_shadow, call, direct_grad, fork_side, ptr, stream, weights_epoch, workspace
from .linalg import DENSE_SIDE_ON, colsum, dense_dgrad, dense_wgrad

E4M3_MAX = 448.0
E5M2_MAX = 57344.0
_FP8_BWD = os.environ.get("DTF_FP8_BWD", "1") != "0"

# state buffer slots (f32, per layer): adjacent pairs are the (s_a, s_b) dequant scales of the three GEMMs
# (forward (x, w), data gradient (w, g), weight gradient (g, x)); X_AMAX / G_AMAX are double-buffered by step
# parity: a quantize pass derives its scale from the previous step's slot and fills the other one, and the GEMM
# that consumes it clears the previous slot for the step after (no scale-update launch)
X_SCALE, W_SCALE, G_SCALE, X_USED, X_AMAX, G_AMAX = range(6)
X_AMAX2, G_AMAX2 = 6, 7
# weights: delayed scaling too (the standard fp8 recipe) — each step's W/W^T quantize pass uses the amax the
# previous step's pass recorded and records its own; the step's weight-gradient GEMM clears the slot just read.
# One launch per weight and step instead of an absmax pass + the quantize pass (False: exact scale; tests).
W_AMAX, W_AMAX2 = 8, 9
_W_DELAYED = True


def quantize(x, scale, amax=None, zero_amax=True):
    q = torch.empty(x.shape, dtype=torch.uint8, device=x.device)
    call("dtf_quant_fp8", ptr(x), ptr(q), x.numel(), ptr(scale), ptr(amax), int(zero_amax), stream())
    return q


def quantize_t(x, scale=None, amax=None, *, fmt=0, pre=None, act=0, rowmajor=True, transposed=True, colsums=False,
               exact_out=None, amax_prev=None, scale_used=None, scale_used2=None):
    """One transposing pass over a [M, N] bf16 matrix (M, N multiples of 64): returns (q [M,N] | None,
    qT [N,M] | None, column-sum partials [ceil(M/256), N] | None). fmt 0 = e4m3, 1 = e5m2. exact_out: compute the
    exact per-tensor scale on the device and store it there (weights); else quantize with `scale` and record
    amax. pre/act: x is the gradient of act(pre) (the activation backward is applied in the pass)."""
    M, N = x.shape
    dev = x.device
    q = torch.empty((M, N), dtype=torch.uint8, device=dev) if rowmajor else None
    qT = torch.empty((N, M), dtype=torch.uint8, device=dev) if transposed else None
    cp = torch.empty((-(-M // 256), N), dtype=F32, device=dev) if colsums else None
    ws = workspace(dev) if exact_out is not None else None
    call("dtf_quant_fp8_t2", ptr(x), ptr(pre), int(act), ptr(q), ptr(qT), ptr(cp), ptr(scale), ptr(amax), M, N,
         int(fmt), int(exact_out is not None), ptr(ws), ptr(exact_out), ptr(amax_prev), ptr(scale_used),
         ptr(scale_used2), stream())
    return q, qT, cp


def gemm_fp8(a, b, scales, out, *, fmt_a=0, out_f32=False, beta=0.0, splitk=1, bias=None, act=0, aux=None,
             zero_slot=None):
    """out[M,N] (=|+=) s0*s1 * a[M,K] . b[N,K]^T (+bias, act with the pre-activation to aux) for fp8 a (fmt_a 0
    e4m3 / 1 e5m2) and e4m3 b (K-contiguous); zero_slot: an f32 the kernel clears (delayed-scaling amax slot)."""
    M, K = a.shape
    N = b.shape[0]
    ws = workspace(a.device) if splitk > 1 else None
    call("dtf_gemm_fp8_ex", ptr(a), ptr(b), ptr(out), ptr(aux), ptr(bias), ptr(scales), M, N, K, a.stride(0),
         b.stride(0), out.stride(0), int(act), int(fmt_a), int(out_f32), float(beta), int(splitk), ptr(ws),
         ws.numel() if ws is not None else 0, ptr(zero_slot), stream())
    return out


_WGRAD_SPLIT_MAX = int(os.environ.get("DTF_FP8_WGRAD_SPLIT_MAX", "4"))


def _wgrad_splits(M, N, K, ws_elems):
    """Split-K factor for the fp8 weight gradient (M x N output, K tokens) on the 4-wave kernel's 256x128 tiles:
    about one round of 1-block/CU tiles, >= 1024 tokens per split, at most _WGRAD_SPLIT_MAX, slabs within the
    workspace. Default 4 since the 4-wave fp8 kernel (its 256x128 tiles leave a 1024 x 1024 weight gradient at 32
    blocks): GPT-2-medium fp8 253.7k / 255.3k tok/s unsplit vs 259.4k / 260.4k with up to 4 splits, interleaved
    (profiles/r5_fp8_w4.txt); with the round-3 8-wave kernel splitting had lost (34.89 ms/step unsplit vs 35.33 with
    2 and 36.25 with 4 splits)."""
    tiles = -(-M // 256) * -(-N // 128)
    s = max(1, min(256 // max(tiles, 1), K // 1024, _WGRAD_SPLIT_MAX))
    while s > 1 and s * M * N > ws_elems:
        s -= 1
    return s


class _Views:
    """The state buffer with its slices cached: every projection call takes ~10 one-element views of it, and building
    a tensor view costs microseconds of host time (a launch-heavy fp8 step is host-bound on a slow CPU)."""
    __slots__ = ("t", "c")

    def __init__(self, t):
        self.t, self.c = t, {}

    def __getitem__(self, k):
        key = (k.start, k.stop) if isinstance(k, slice) else k
        v = self.c.get(key)
        if v is None:
            v = self.c[key] = self.t[k]
        return v


class _Fp8State:
    def __init__(self, dev):
        self.buf = torch.zeros(10, dtype=F32, device=dev)
        self.buf[W_SCALE] = 1.0
        self.bv = _Views(self.buf)
        self.x_ready = False
        self.g_ready = False
        self.tx = 0  # forward / backward / weight step counters: parity of the double-buffered amax slots
        self.tg = 0
        self.tw = 0
        self.w_ready = False
        self.w_prev = None  # the weight amax slot this step's pass read (cleared by this step's weight gradient)
        self.wq = self.wqT = None
        self.w_key = None
        # fp8 operands written by the neighbouring layer's GEMM epilogue (gemm256.hip q8 outputs), matched by the
        # data pointer of the placeholder that stands for the bf16 tensor nobody wrote:
        self.pending_x = None  # (ptr, xq, xqT, amax slot to clear, producer state, producer pre, producer act)
        self.pending_g = None  # (ptr, dzq, dzqT, column-sum partials, amax slot to clear)


def _state(layer, dev):
    st = getattr(layer, "_fp8", None)
    if st is None:
        st = _Fp8State(dev)
        object.__setattr__(layer, "_fp8", st)
    return st


def _weight_fp8(st, w, need_t):
    key = (weights_epoch(), w._version, need_t)
    if st.wq is not None and st.w_key == key:
        return st.wq, st.wqT
    w16 = bf16_shadow(w)
    N, K = w16.shape
    buf = st.bv
    if need_t and _W_DELAYED and not torch.cuda.is_current_stream_capturing():
        cur, prev = (W_AMAX, W_AMAX2) if st.tw % 2 == 0 else (W_AMAX2, W_AMAX)
        st.tw += 1
        if not st.w_ready:  # bootstrap: exact scale once, recording the amax the next step scales with
            st.wq, st.wqT, _ = quantize_t(w16, amax=buf[cur:cur + 1], exact_out=buf[W_SCALE:W_SCALE + 1])
            st.w_ready = True
            st.w_prev = None
        else:
            st.wq, st.wqT, _ = quantize_t(w16, buf[W_SCALE:W_SCALE + 1], buf[cur:cur + 1],
                                          amax_prev=buf[prev:prev + 1], scale_used=buf[W_SCALE:W_SCALE + 1])
            st.w_prev = prev
    elif need_t:
        # exact per-tensor scale (amax/448) computed on the device; W and W^T from one transposing pass
        st.wq, st.wqT, _ = quantize_t(w16, exact_out=st.bv[W_SCALE:W_SCALE + 1])
    else:
        if st.wq is None or st.wq.shape != w16.shape:
            st.wq = torch.empty(w16.shape, dtype=torch.uint8, device=w16.device)
        ws = workspace(w16.device)
        call("dtf_quant_fp8_exact", ptr(w16), ptr(st.wq), w16.numel(), ptr(st.bv[W_SCALE:W_SCALE + 1]), ptr(ws),
             stream())
        st.wqT = None
    st.w_key = key
    return st.wq, st.wqT


def _fp8_bwd_ok(M, K, N):
    return _FP8_BWD and M % 128 == 0 and K % 128 == 0 and N % 128 == 0


# Producer-side quantization (_FUSE, on; tests switch it off to compare): a GELU projection whose only consumer is another fp8
# projection (GPT-2's FFN1 -> FFN2, linked by _Proj.fp8_next) writes FFN2's e4m3 input and its transpose from its own
# GEMM epilogue, and FFN2's data-gradient GEMM writes FFN1's e5m2 gradient (GELU backward applied), its transpose and
# the bias-gradient column sums from its epilogue: the bf16 GELU output and the bf16 gradient of it are never
# written, and two quantize passes per layer and step leave the critical stream. Delayed scaling is unchanged (the
# same amax slots, parities and scale publication as the quantize pass).
_FUSE = True
_FUSE_BWD = True  # the gradient half (FFN2's dgrad writes FFN1's e5m2 dZ)


def _placeholder(shape, dev):
    """A stand-in for a bf16 activation / gradient that only exists in fp8 (its consumer finds the fp8 copies by
    this tensor's data pointer): one element, expanded (zero strides, no storage of the full size)."""
    return torch.empty(1, dtype=BF16, device=dev).expand(*shape)


def _gemm_q8(a, b, scales, out, *, fmt_a, q8, q8T, q8col, q8fmt, q8buf, q8scale, q8cur, q8prev, q8used2=None,
             bias=None, act=0, aux=None, dact_src=None, dact=0, zero_slot=None):
    """gemm_fp8 whose epilogue also writes fp8 copies of its output (dtf_gemm_fp8_q8); False when the pipelined
    kernel cannot take the shape (nothing was launched)."""
    M, Kd = a.shape
    N = b.shape[0]
    rc = K().dtf_gemm_fp8_q8(ptr(a), ptr(b), ptr(out), ptr(aux), ptr(bias), ptr(scales), M, N, Kd, a.stride(0),
                             b.stride(0), int(act), int(fmt_a), ptr(dact_src), int(dact), ptr(zero_slot), ptr(q8),
                             ptr(q8T), ptr(q8col), int(q8fmt), ptr(q8buf[q8scale:q8scale + 1]),
                             ptr(q8buf[q8cur:q8cur + 1]), ptr(q8buf[q8prev:q8prev + 1]),
                             ptr(q8buf[q8scale:q8scale + 1]), ptr(q8used2), stream())
    if rc == -6:
        return False
    if rc != 0:
        raise RuntimeError(f"dtf_gemm_fp8_q8 failed with status {rc}")
    return True


class _DenseFP8(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, act, st, nxt=None):
        shp = x.shape
        N = w.shape[0]
        buf = st.bv
        pend, st.pending_x = st.pending_x, None
        ctx.src = None
        if pend is not None and x.data_ptr() == pend[0]:
            # x exists only in fp8: the producing layer's epilogue wrote it (and its transpose) with our scale
            xq, xqT, prev = pend[1], pend[2], pend[3]
            M, K = xq.shape
            ctx.src = pend[4:]  # (producer state, its pre-activation, its activation): the fused dgrad target
            pre = torch.empty((M, N), dtype=BF16, device=x.device) if act else None
            wq, wqT = _weight_fp8(st, w, True)
            y = torch.empty((M, N), dtype=BF16, device=x.device)
            gemm_fp8(xq, wq, buf[X_SCALE:X_SCALE + 2], y, bias=b, act=act, aux=pre, zero_slot=buf[prev:prev + 1])
            return _DenseFP8._finish_fwd(ctx, True, xqT, w, pre, st, b, act, shp, (M, K, N), y)
        x2 = x.reshape(-1, shp[-1]).contiguous()
        M, K = x2.shape
        fbwd = _fp8_bwd_ok(M, K, N)
        if not st.x_ready:  # bootstrap the delayed activation scale once
            buf[X_SCALE:X_SCALE + 1].copy_(x2.abs().amax().float().clamp_min(1e-12) / E4M3_MAX)
            st.x_ready = True
        xs = buf[X_SCALE:X_SCALE + 1]
        pre = torch.empty((M, N), dtype=BF16, device=x.device) if act else None
        nst = _state(nxt, x.device) if nxt is not None else None
        if (nst is not None and _FUSE and fbwd and act and nst.x_ready and M % 256 == 0
                and not torch.cuda.is_current_stream_capturing()):
            # our output feeds only the next fp8 projection: write its e4m3 operand (+ transpose) instead of bf16
            cur, prev = (X_AMAX, X_AMAX2) if st.tx % 2 == 0 else (X_AMAX2, X_AMAX)
            ncur, nprev = (X_AMAX, X_AMAX2) if nst.tx % 2 == 0 else (X_AMAX2, X_AMAX)
            xq, xqT, _ = quantize_t(x2, xs, buf[cur:cur + 1], amax_prev=buf[prev:prev + 1], scale_used=xs,
                                    scale_used2=buf[X_USED:X_USED + 1])
            st.tx += 1
            wq, wqT = _weight_fp8(st, w, True)
            yq = torch.empty((M, N), dtype=torch.uint8, device=x.device)
            yqT = torch.empty((N, M), dtype=torch.uint8, device=x.device)
            nb = nst.bv
            if _gemm_q8(xq, wq, buf[X_SCALE:X_SCALE + 2], None, fmt_a=0, q8=yq, q8T=yqT, q8col=None, q8fmt=0,
                        q8buf=nb, q8scale=X_SCALE, q8cur=ncur, q8prev=nprev, q8used2=nb[X_USED:X_USED + 1],
                        bias=b, act=act, aux=pre, zero_slot=buf[prev:prev + 1]):
                nst.tx += 1
                y = _placeholder((M, N), x.device)
                nst.pending_x = (y.data_ptr(), yq, yqT, nprev, st, pre, act)
                return _DenseFP8._finish_fwd(ctx, True, xqT, w, pre, st, b, act, shp, (M, K, N), y)
            y = torch.empty((M, N), dtype=BF16, device=x.device)  # (shape not taken by the pipelined kernel)
            gemm_fp8(xq, wq, buf[X_SCALE:X_SCALE + 2], y, bias=b, act=act, aux=pre, zero_slot=buf[prev:prev + 1])
            return _DenseFP8._finish_fwd(ctx, True, xqT, w, pre, st, b, act, shp, (M, K, N), y)
        y = torch.empty((M, N), dtype=BF16, device=x.device)
        if fbwd and not torch.cuda.is_current_stream_capturing():
            # delayed scaling folded into the quantize pass (amax slots double-buffered by step parity)
            cur, prev = (X_AMAX, X_AMAX2) if st.tx % 2 == 0 else (X_AMAX2, X_AMAX)
            st.tx += 1
            xq, xqT, _ = quantize_t(x2, xs, buf[cur:cur + 1], amax_prev=buf[prev:prev + 1], scale_used=xs,
                                    scale_used2=buf[X_USED:X_USED + 1])
            wq, wqT = _weight_fp8(st, w, True)
            gemm_fp8(xq, wq, buf[X_SCALE:X_SCALE + 2], y, bias=b, act=act, aux=pre, zero_slot=buf[prev:prev + 1])
        else:
            xa = buf[X_AMAX:X_AMAX + 1]
            if fbwd:
                xq, xqT, _ = quantize_t(x2, xs, xa)
            else:
                xq, xqT = quantize(x2, xs, xa, zero_amax=False), None
            wq, wqT = _weight_fp8(st, w, fbwd)
            call("dtf_gemm_fp8", ptr(xq), ptr(wq), ptr(y), ptr(pre), ptr(b), ptr(buf[X_SCALE:X_SCALE + 2]), M, N, K,
                 K, K, N, int(act), -1, stream())
            # next step's x scale from this pass's amax; the scale this pass used is kept for the weight gradient
            call("dtf_fp8_update_scale2", ptr(xa), ptr(xs), ptr(buf[X_USED:X_USED + 1]), E4M3_MAX, 0.0, stream())
        return _DenseFP8._finish_fwd(ctx, fbwd, xqT if fbwd else x2, w, pre, st, b, act, shp, (M, K, N), y)

    @staticmethod
    def _finish_fwd(ctx, fbwd, xs, w, pre, st, b, act, shp, MKN, y):
        ctx.fbwd = fbwd
        ctx.save_for_backward(xs, w, pre)  # xs: x^T in e4m3 (fp8 backward) or the bf16 x
        ctx.st = st
        ctx.b_param = b
        ctx.act = act
        ctx.has_b = b is not None
        ctx.shp = shp
        ctx.MKN = MKN
        return y.reshape(*shp[:-1], MKN[2])

    @staticmethod
    def backward(ctx, dy):
        if not ctx.fbwd:
            return _DenseFP8._backward_bf16(ctx, dy)
        xqT, w, pre = ctx.saved_tensors
        st, (M, K, N) = ctx.st, ctx.MKN
        buf = st.bv
        gs, ga = buf[G_SCALE:G_SCALE + 1], buf[G_AMAX:G_AMAX + 1]
        need_dx, need_dw = ctx.needs_input_grad[0], ctx.needs_input_grad[1]
        need_db = ctx.has_b and ctx.needs_input_grad[2]
        gpend, st.pending_g = st.pending_g, None
        fused_in = gpend is not None and dy.data_ptr() == gpend[0] and need_dx
        if not fused_in:
            dy2 = dy.reshape(-1, N).to(BF16).contiguous()
            if not st.g_ready:  # bootstrap the delayed gradient scale once (GELU' <= 1.13)
                gs.copy_(dy2.abs().amax().float().clamp_min(1e-30) * (1.2 if ctx.act else 1.0) / E5M2_MAX)
                st.g_ready = True
        folded = need_dx and not torch.cuda.is_current_stream_capturing()
        prev = None
        if fused_in:  # the consumer's data-gradient epilogue quantized our gradient (act backward applied)
            dzq, dzqT, cp, prev = gpend[1], gpend[2], gpend[3], gpend[4]
        elif folded:  # delayed gradient scaling folded into the quantize pass (see forward)
            cur, prev = (G_AMAX, G_AMAX2) if st.tg % 2 == 0 else (G_AMAX2, G_AMAX)
            st.tg += 1
            dzq, dzqT, cp = quantize_t(dy2, gs, buf[cur:cur + 1], fmt=1, pre=pre if ctx.act else None, act=ctx.act,
                                       rowmajor=True, transposed=need_dw, colsums=need_db,
                                       amax_prev=buf[prev:prev + 1], scale_used=gs)
        else:
            dzq, dzqT, cp = quantize_t(dy2, gs, ga, fmt=1, pre=pre if ctx.act else None, act=ctx.act,
                                       rowmajor=need_dx, transposed=need_dw, colsums=need_db)
        dx = dw = db = None
        if need_dx:
            _, wqT = _weight_fp8(st, w, True)
            src, ctx.src = ctx.src, None
            dx = None
            if (src is not None and _FUSE_BWD and folded and src[0] is not None and src[0].g_ready and src[2]
                    and M % 256 == 0):
                # our input came from the producer's fp8 epilogue: quantize ITS gradient here (the activation
                # backward from its saved pre-activation, e5m2 + transpose + bias-gradient column partials)
                pst, ppre, pact = src
                pb = pst.bv
                pcur, pprev = (G_AMAX, G_AMAX2) if pst.tg % 2 == 0 else (G_AMAX2, G_AMAX)
                gq = torch.empty((M, K), dtype=torch.uint8, device=dy.device)
                gqT = torch.empty((K, M), dtype=torch.uint8, device=dy.device)
                gcp = torch.empty((M // 128, K), dtype=F32, device=dy.device)
                if _gemm_q8(dzq, wqT, buf[W_SCALE:W_SCALE + 2], None, fmt_a=1, q8=gq, q8T=gqT, q8col=gcp, q8fmt=1,
                            q8buf=pb, q8scale=G_SCALE, q8cur=pcur, q8prev=pprev, dact_src=ppre, dact=pact,
                            zero_slot=buf[prev:prev + 1]):
                    pst.tg += 1
                    dx = _placeholder((M, K), dy.device)
                    pst.pending_g = (dx.data_ptr(), gq, gqT, gcp, pprev)
                    dx = dx.reshape(ctx.shp)
            if dx is None:
                dx = torch.empty((M, K), dtype=BF16, device=dy.device)
                gemm_fp8(dzq, wqT, buf[W_SCALE:W_SCALE + 2], dx, fmt_a=1,  # scales (s_w, s_g)
                         zero_slot=buf[prev:prev + 1] if folded else None)
                dx = dx.reshape(ctx.shp)
        tw = direct_grad(w) if need_dw else None
        tb = direct_grad(ctx.b_param) if need_db else None
        # arena-accumulated weight / bias gradients go to the side stream (off the dgrad critical path)
        side = (fork_side(dy.device, dzqT, xqT, cp, st.buf) if (tw is not None and DENSE_SIDE_ON)
                else contextlib.nullcontext())
        with side:
            if need_dw:  # dW[N, K] (+)= dZ^T X over the M tokens; inside Model.train_step straight into the arena
                wprev, st.w_prev = st.w_prev, None
                out = tw if tw is not None else torch.empty((N, K), dtype=F32, device=dy.device)
                sk = _wgrad_splits(N, K, M, workspace(dy.device).numel())
                gemm_fp8(dzqT, xqT, buf[G_SCALE:G_SCALE + 2], out, fmt_a=1, out_f32=True,
                         beta=1.0 if tw is not None else 0.0, splitk=sk,  # scales (s_g, s_x used)
                         zero_slot=None if wprev is None else buf[wprev:wprev + 1])
                dw = None if tw is not None else out
            if need_db:
                out = tb if tb is not None else torch.empty(N, dtype=F32, device=dy.device)
                call("dtf_reduce_rows", ptr(cp), N, cp.shape[0], N, ptr(out), int(tb is not None), stream())
                db = None if tb is not None else out
            if not folded:
                # next step's gradient scale: on the stream of the last reader of this step's scale (the weight
                # gradient), which was forked after the data gradient was issued
                call("dtf_fp8_update_scale2", ptr(ga), ptr(gs), None, E5M2_MAX, 0.0, stream())
        return dx, dw, db, None, None, None

    @staticmethod
    def _backward_bf16(ctx, dy):
        x2, w, pre = ctx.saved_tensors
        N = w.shape[0]
        dz = dy.reshape(-1, N).to(BF16).contiguous()
        if ctx.act:
            g = torch.empty_like(dz)
            call("dtf_act", ptr(pre), ptr(dz), ptr(g), g.numel(), ctx.act, 1, stream())
            dz = g
        dx = dense_dgrad(dz, bf16_shadow(w)).reshape(ctx.shp) if ctx.needs_input_grad[0] else None
        dw = db = None
        if ctx.needs_input_grad[1]:  # inside Model.train_step: accumulate into the arena gradient directly
            tw = direct_grad(w)
            if tw is not None:
                dense_wgrad(dz, x2, out=tw)
            else:
                dw = dense_wgrad(dz, x2)
        if ctx.has_b and ctx.needs_input_grad[2]:
            tb = direct_grad(ctx.b_param)
            if tb is not None:
                colsum(dz, out=tb, accumulate=True)
            else:
                db = colsum(dz)
        return dx, dw, db, None, None, None


def dense_fp8(x, w, b, activation, layer, next_layer=None):
    """next_layer: the fp8 projection that is the ONLY consumer of this one's output (its operands may then be
    written by this layer's epilogue; see _FUSE)."""
    from .linalg import act_code
    a = act_code(activation)
    st = _state(layer, x.device)
    return _DenseFP8.apply(x if x.dtype == BF16 else x.to(BF16), w, b, a, st, next_layer)
