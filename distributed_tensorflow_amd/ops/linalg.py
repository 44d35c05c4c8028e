"""MatMul / Dense (Linear) / batched matmul on the gfx950 MFMA GEMM (csrc/kernels/gemm.hip).

TF's MatMul + BiasAdd (+ activation) and their gradients.
On GPU every product runs on the hand-written MFMA kernel; on CPU the same
function evaluates the f32 reference so the API works device-agnostically.
"""
from __future__ import annotations

import torch

from ._util import (BF16, F32, SIDE_STREAM_ON, IntOut, K, bf16_shadow, call, direct_grad, fork_side, on_gpu, ptr,
                    stream, workspace)

ACT_NONE, ACT_RELU, ACT_GELU = 0, 1, 2
_ACTS = {None: 0, "linear": 0, "relu": 1, "gelu": 2}


def act_code(act):
    if isinstance(act, int):
        return act
    return _ACTS[act]


def gemm(a, b, *, a_kouter=False, b_kouter=False, out=None, out_dtype=BF16, bias=None, act=0, alpha=1.0,
         beta=0.0, stats=None, aux=None, splitk=0, tile=-1):
    """C[m,n] = alpha * sum_k A(m,k) B(n,k) + beta*C  (+bias[n], act).

    A is [M,K] (or [K,M] if a_kouter), B is [N,K] (or [K,N] if b_kouter); 2-D or
    batched 3-D (leading batch dim). bf16 inputs; C bf16 or f32.
    """
    assert a.dtype == BF16 and b.dtype == BF16, "gemm operands must be bf16"
    padded = _pad_operands(a, b, a_kouter, b_kouter)
    if padded is not None:
        a2, b2, M, N = padded
        o = gemm(a2, b2, a_kouter=a_kouter, b_kouter=b_kouter, out_dtype=out_dtype if out is None else out.dtype,
                 bias=None if bias is None else torch.nn.functional.pad(bias, (0, b2.shape[-1 if b_kouter else -2]
                                                                               - N)),
                 act=act, alpha=alpha, splitk=splitk, tile=tile)
        o = o[..., :M, :N]
        if stats is not None:
            y = o.float()
            red = tuple(range(y.dim() - 1))
            stats[:N] += y.sum(red)
            stats[N:] += (y * y).sum(red)
        if aux is not None:
            raise NotImplementedError("aux output with padded gemm")
        if out is None:
            return o.contiguous()
        if beta != 0:
            out.mul_(beta).add_(o.to(out.dtype))
        else:
            out.copy_(o)
        return out
    batched = a.dim() == 3
    if batched:
        bt = a.shape[0]
        M, K = (a.shape[2], a.shape[1]) if a_kouter else (a.shape[1], a.shape[2])
        N = b.shape[2] if b_kouter else b.shape[1]
    else:
        bt = 1
        M, K = (a.shape[1], a.shape[0]) if a_kouter else (a.shape[0], a.shape[1])
        N = b.shape[1] if b_kouter else b.shape[0]
    if out is None:
        shape = (bt, M, N) if batched else (M, N)
        out = (torch.zeros if beta != 0 else torch.empty)(shape, dtype=out_dtype, device=a.device)
    lda = a.stride(-2)
    ldb = b.stride(-2)
    ldc = out.stride(-2)
    sA = a.stride(0) if batched else 0
    sB = b.stride(0) if batched else 0
    sC = out.stride(0) if batched else 0
    part = rows = None
    ws = workspace(a.device) if out.dtype == F32 else None
    if stats is not None:  # kernel writes per-M-tile partial rows; reduce them here
        part = torch.empty(((M + 63) // 64) * 2 * N, dtype=F32, device=a.device)
        rows = IntOut()
        splitk = 1
    call("dtf_gemm", ptr(a), ptr(b), ptr(out), ptr(aux), ptr(bias), ptr(part), rows.addr if rows else None, M, N, K,
         lda, ldb, ldc, int(a_kouter), int(b_kouter), bt, sA, sB, sC, float(alpha), float(beta), int(act),
         int(out.dtype == F32), int(splitk), int(tile), ptr(ws), ws.numel() if ws is not None else 0, stream())
    if stats is not None:
        stats += part[:rows.value * 2 * N].view(rows.value, 2 * N).sum(0)
    return out


def _pad_operands(a, b, a_kouter, b_kouter):
    """Zero-pad to the kernel's alignment (K%8, M%8 / N%8 for K-outer operands, N%4); None if aligned."""
    if a_kouter:
        K, M = a.shape[-2], a.shape[-1]
    else:
        M, K = a.shape[-2], a.shape[-1]
    if b_kouter:
        N = b.shape[-1]
    else:
        N = b.shape[-2]
    Kp = -(-K // 8) * 8
    Mp = -(-M // 8) * 8 if a_kouter else M
    Np = -(-N // 8) * 8 if b_kouter else -(-N // 4) * 4
    if (Kp, Mp, Np) == (K, M, N):
        return None
    F = torch.nn.functional
    if a_kouter:
        a2 = F.pad(a, (0, Mp - M, 0, Kp - K))
    else:
        a2 = F.pad(a, (0, Kp - K))
    if b_kouter:
        b2 = F.pad(b, (0, Np - N, 0, Kp - K))
    else:
        b2 = F.pad(b, (0, Kp - K, 0, Np - N))
    return a2.contiguous(), b2.contiguous(), M, N


def colsum(x2d, out=None, accumulate=False):
    """BiasAddGrad: column sums of a bf16 [M,N] matrix into f32 [N]."""
    M, N = x2d.shape
    if N % 8:
        r = x2d.float().sum(0)
        if out is None:
            return r
        return out.add_(r) if accumulate else out.copy_(r)
    if out is None:
        out = torch.empty(N, dtype=F32, device=x2d.device)
    ws = workspace(x2d.device)
    call("dtf_colsum", ptr(x2d), M, N, ptr(out), int(accumulate), ptr(ws), ws.numel(), stream())
    return out


# Dense weight gradients on the side stream (with SIDE_STREAM_ON).
# Every dense GEMM runs on the hand-written kernels (gemm.hip -> gemm_w4.hip for the 256-row tiles); the round-4
# hipBLASLt routes for the plain projections were removed in round 5.
DENSE_SIDE_ON = SIDE_STREAM_ON
_SPLIT_DGRAD_K = 8192  # data gradients over a K this long with few output tiles: split-K f32 route (0 disables)


def dense_dgrad(dz, w16, acc=None):
    """dX[T, in] = dZ[T, out] W[out, in] (bf16); with `acc` (another gradient of the same input, [T, in], parked on
    a ResidualGradLink: no other reader) the GEMM adds it in its store pass and returns it — no separate add pass,
    the same values as the GEMM followed by an elementwise add."""
    M, K, N = dz.shape[0], dz.shape[1], w16.shape[1]
    if acc is None and _SPLIT_DGRAD_K and K >= _SPLIT_DGRAD_K and -(-M // 128) * -(-N // 128) < 256 and dz.is_cuda:
        # few output tiles over a long K (BERT's MLM decoder: 2432 x 768 over the 30k vocabulary): split-K f32 slabs
        # on the wide tiles instead of one bf16 pass of small tiles, then one rounding to bf16 (BERT-base +1.7%)
        o = gemm(dz, w16, b_kouter=True, out_dtype=F32)
        out = torch.empty((M, N), dtype=BF16, device=dz.device)
        call("dtf_cast_f32_bf16", ptr(o), ptr(out), o.numel(), stream())
        return out
    if acc is None:
        return gemm(dz, w16, b_kouter=True)
    return gemm(dz, w16, b_kouter=True, out=acc, beta=1.0)


def dense_wgrad_bias(dz, x2, out, bias_out):
    """dW += dZ^T X and db += column sums of dZ in ONE 4-wave GEMM launch (the bias gradient from the dZ fragments the
    weight-gradient kernel already holds: gemm.hip dtf_gemm_wgrad_bias); False when that kernel cannot take the shape
    (nothing ran: use dense_wgrad + colsum)."""
    if not (dz.is_cuda and out.dtype == F32 and out.is_contiguous() and bias_out.is_contiguous()):
        return False
    T, M = dz.shape
    N = x2.shape[1]
    ws = workspace(dz.device)
    rc = K().dtf_gemm_wgrad_bias(ptr(dz), ptr(x2), ptr(out), ptr(bias_out), M, N, T, dz.stride(0), x2.stride(0), N,
                                 1.0, ptr(ws), ws.numel(), stream())
    return rc == 0


def dense_wgrad(dz, x2, out=None):
    """dW[out, in] = dZ^T X in f32; accumulated into `out` (an arena gradient view) when given."""
    if out is not None:
        return gemm(dz, x2, a_kouter=True, b_kouter=True, out=out, beta=1.0)
    return gemm(dz, x2, a_kouter=True, b_kouter=True, out_dtype=F32)


def _act_ref(x, act):
    if act == ACT_RELU:
        return torch.relu(x)
    if act == ACT_GELU:
        return torch.nn.functional.gelu(x, approximate="tanh")
    return x


class _ActSource:
    """Attached to the output of a Dense layer with an activation (the pre-activation and the activation code): a
    consuming Dense layer that is the output's only reader applies the activation backward inside its own
    data-gradient GEMM epilogue (gemm_dact), and the producer then skips its activation-backward pass — the
    gradient of the activation output is never written (cf. ops.conv._BNSource for BatchNorm)."""
    __slots__ = ("pre", "act", "consumers", "fused_ptr", "__weakref__")

    def __init__(self, pre, act):
        self.pre, self.act = pre, act
        self.consumers = 0
        self.fused_ptr = None


_FUSE_DACT = True
# the bias gradient of an arena-accumulated Dense layer inside its weight-gradient GEMM (dense_wgrad_bias) instead of a
# separate column-sum pass over dZ
_FUSE_BIAS_GRAD = True


class _DenseFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, act, link=None, tag_act=False):
        # x: [..., in] bf16 ; w: [out, in] f32 master ; b: [out] f32 or None
        # link: ops.conv.ResidualGradLink whose parked gradient of x the data-gradient GEMM adds in
        # tag_act: the caller guarantees the output is read by ONE Dense layer only (e.g. FFN1 -> FFN2), which may
        # then fuse this layer's activation backward into its data-gradient GEMM (_ActSource)
        ctx.link = link
        in_src = getattr(x, "_dtf_actsrc", None)
        if in_src is not None:
            in_src.consumers += 1
        ctx.in_src = in_src
        shp = x.shape
        x2 = x.reshape(-1, shp[-1])
        if not x2.is_contiguous():
            x2 = x2.contiguous()
        w16 = bf16_shadow(w)
        pre = torch.empty((x2.shape[0], w.shape[0]), dtype=BF16, device=x.device) if act else None
        y = gemm(x2, w16, bias=b, act=act, aux=pre)
        ctx.save_for_backward(x2, w, pre)
        ctx.act = act
        ctx.has_b = b is not None
        ctx.b_param = b
        ctx.shp = shp
        out = y.reshape(*shp[:-1], w.shape[0])
        ctx.src = None
        if act and tag_act and _FUSE_DACT and pre is not None:
            ctx.src = _ActSource(pre, act)
            out._dtf_actsrc = ctx.src
        return out

    @staticmethod
    def backward(ctx, dy):
        x2, w, pre = ctx.saved_tensors
        dy2 = dy.reshape(-1, w.shape[0])
        if dy2.dtype != BF16:
            dy2 = dy2.to(BF16)
        dy2 = dy2.contiguous()
        src = ctx.src
        ctx.src = None
        if ctx.act and not (src is not None and src.fused_ptr == dy2.data_ptr()):
            dz = torch.empty_like(dy2)
            call("dtf_act", ptr(pre), ptr(dy2), ptr(dz), dz.numel(), ctx.act, 1, stream())
        else:
            dz = dy2  # (the consumer's data-gradient GEMM already applied act')
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            # dx[t,i] = sum_o dz[t,o] W[o,i]  -> B stored [K=out][N=in] (k-outer)
            acc = ctx.link.take()[0] if ctx.link is not None else None
            isrc = ctx.in_src
            ctx.in_src = None
            if (acc is None and isrc is not None and isrc.consumers == 1
                    and isrc.pre.shape == (dz.shape[0], w.shape[1])):
                # the producer's activation backward in this GEMM's epilogue
                dx = torch.empty((dz.shape[0], w.shape[1]), dtype=BF16, device=dz.device)
                w16 = bf16_shadow(w)
                call("dtf_gemm_dact", ptr(dz), ptr(w16), ptr(dx), ptr(isrc.pre), int(isrc.act), dz.shape[0],
                     w.shape[1], w.shape[0], dz.stride(0), w16.stride(0), dx.stride(0), 0, 1, stream())
                isrc.fused_ptr = dx.data_ptr()
            else:
                dx = dense_dgrad(dz, bf16_shadow(w), None if acc is None else acc.reshape(dz.shape[0], -1))
            dx = dx.reshape(ctx.shp)
        tw = direct_grad(w) if ctx.needs_input_grad[1] else None
        tb = direct_grad(ctx.b_param) if (ctx.has_b and ctx.needs_input_grad[2]) else None
        if tw is not None and tw.dim() == 2 and DENSE_SIDE_ON and dz.is_cuda:
            # arena-accumulated weight / bias gradients on the side stream: off the dgrad critical path, and their
            # blocks fill the partial last wave of the data-gradient GEMMs (and vice versa)
            with fork_side(dz.device, dz, x2):
                if not (tb is not None and _FUSE_BIAS_GRAD and dense_wgrad_bias(dz, x2, tw, tb)):
                    dense_wgrad(dz, x2, out=tw)
                    if tb is not None:
                        colsum(dz, out=tb, accumulate=True)
            if ctx.has_b and ctx.needs_input_grad[2] and tb is None:
                db = colsum(dz)
            ctx.link = None
            return dx, dw, db, None, None, None
        if ctx.needs_input_grad[1]:
            # dW[o,i] = sum_t dz[t,o] x[t,i]  -> both operands k-outer, f32 out; inside Model.train_step
            # accumulated straight into the arena gradient (beta = 1) instead of returned
            if tw is not None and tw.dim() == 2:
                dense_wgrad(dz, x2, out=tw)
            else:
                dw = dense_wgrad(dz, x2)
        if ctx.has_b and ctx.needs_input_grad[2]:
            if tb is not None:
                colsum(dz, out=tb, accumulate=True)
            else:
                db = colsum(dz)
        ctx.link = None
        return dx, dw, db, None, None, None


def dense(x, w, b=None, act=None, link=None, tag_act=False):
    """y = act(x @ w^T + b); w is [out, in] (f32 master variable). link: ops.conv.ResidualGradLink joining x's
    gradient from a residual connection into this layer's data-gradient GEMM. tag_act: y feeds exactly one Dense
    layer, which then applies act' inside its data-gradient GEMM (see _ActSource)."""
    a = act_code(act)
    if on_gpu(x):
        if x.dtype != BF16:
            x = x.to(BF16)
        return _DenseFn.apply(x, w, b, a, link, bool(tag_act))
    y = torch.nn.functional.linear(x.to(w.dtype), w, b)
    return _act_ref(y, a)


class _BMMFn(torch.autograd.Function):
    """Batched C = A @ B^T (nt=True) or A @ B (nt=False) for bf16 [b, m, k] tensors."""

    @staticmethod
    def forward(ctx, a, b, nt, alpha):
        a = a.contiguous()
        b = b.contiguous()
        ctx.save_for_backward(a, b)
        ctx.nt = nt
        ctx.alpha = alpha
        return gemm(a, b, b_kouter=not nt, alpha=alpha)

    @staticmethod
    def backward(ctx, dc):
        a, b = ctx.saved_tensors
        dc = dc.to(BF16).contiguous()
        al = ctx.alpha
        if ctx.nt:  # C = A B^T : dA = dC B ; dB = dC^T A
            da = gemm(dc, b, b_kouter=True, alpha=al)
            db = gemm(dc, a, a_kouter=True, b_kouter=True, alpha=al)
        else:  # C = A B : dA = dC B^T ; dB = A^T dC
            da = gemm(dc, b, alpha=al)
            db = gemm(a, dc, a_kouter=True, b_kouter=True, alpha=al)
        return da, db, None, None


def bmm(a, b, transpose_b=False, alpha=1.0):
    if on_gpu(a):
        return _BMMFn.apply(a.to(BF16), b.to(BF16), bool(transpose_b), float(alpha))
    bb = b.transpose(-1, -2) if transpose_b else b
    return alpha * torch.matmul(a, bb)


def matmul(a, b, transpose_a=False, transpose_b=False):
    """tf.linalg.matmul-like entry point (2-D or batched)."""
    if transpose_a:
        a = a.transpose(-1, -2)
    if a.dim() == 2 and b.dim() == 2:
        return bmm(a.unsqueeze(0), b.unsqueeze(0), transpose_b=transpose_b)[0] if on_gpu(a) else (
            a @ (b.transpose(-1, -2) if transpose_b else b))
    return bmm(a, b, transpose_b=transpose_b)
