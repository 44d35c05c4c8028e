"""FusedBatchNorm (NHWC) and LayerNorm ops (csrc/kernels/norm.hip), with CPU references."""
from __future__ import annotations

import torch

from ._util import BF16, F32, SIDE_STREAM_ON, IntOut, call, direct_grad, fork_side, on_gpu, ptr, stream, workspace
from .nn import take_pending


def batch_norm_ref(y, gamma, beta, rmean, rvar, momentum, eps, training):
    """f32 reference of training/inference BN over all but the last (channel) axis."""
    yf = y.float()
    red = tuple(range(yf.dim() - 1))
    if training:
        mean = yf.mean(dim=red)
        var = yf.var(dim=red, unbiased=False)
        if rmean is not None:
            n = yf.numel() // yf.shape[-1]
            with torch.no_grad():
                rmean.mul_(momentum).add_(mean.detach() * (1 - momentum))
                rvar.mul_(momentum).add_(var.detach() * (n / max(n - 1, 1)) * (1 - momentum))
    else:
        mean, var = rmean, rvar
    out = (yf - mean) * torch.rsqrt(var + eps)
    if gamma is not None:
        out = out * gamma
    if beta is not None:
        out = out + beta
    return out


class _BNFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, gamma, beta, res, rmean, rvar, relu, momentum, eps, training):
        x = x.contiguous()
        C = x.shape[-1]
        M = x.numel() // C
        work = torch.empty(4 * C, dtype=F32, device=x.device)
        scale, shift, mean, invstd = work[:C], work[C:2 * C], work[2 * C:3 * C], work[3 * C:]
        if training:
            part = torch.empty(1024 * 2 * C, dtype=F32, device=x.device)
            rows = IntOut()
            call("dtf_bn_stats", ptr(x), M, C, ptr(part), rows.addr, stream())
            call("dtf_bn_finalize", ptr(part), rows.value, ptr(gamma), ptr(beta), ptr(rmean), ptr(rvar), M, C,
                 float(momentum), float(eps), ptr(scale), ptr(shift), ptr(mean), ptr(invstd), stream())
        else:
            call("dtf_bn_infer_coeff", ptr(gamma), ptr(beta), ptr(rmean), ptr(rvar), C, float(eps), ptr(scale),
                 ptr(shift), stream())
        out = torch.empty_like(x)
        if res is not None:
            res = res.to(BF16).contiguous()
        mbits = torch.empty(M * C // 8, dtype=torch.uint8, device=x.device) if relu else None
        call("dtf_bn_apply", ptr(x), ptr(scale), ptr(shift), ptr(res), ptr(out), M, C, int(relu), ptr(mbits),
             None, None, stream())
        ctx.save_for_backward(x, gamma, mbits, mean, invstd)
        ctx.relu = relu
        ctx.has_res = res is not None
        return out

    @staticmethod
    def backward(ctx, dout):
        x, gamma, mbits, mean, invstd = ctx.saved_tensors
        C = x.shape[-1]
        M = x.numel() // C
        dout = dout.to(BF16).contiguous()
        dx = torch.empty_like(x)
        dres = torch.empty_like(x) if (ctx.has_res and ctx.relu) else None
        dgamma = torch.empty(C, dtype=F32, device=x.device)
        dbeta = torch.empty(C, dtype=F32, device=x.device)
        work = torch.empty((2 * 1024 + 3) * C, dtype=F32, device=x.device)
        call("dtf_bn_bwd", ptr(dout), None, ptr(mbits), ptr(x), ptr(mean), ptr(invstd), ptr(gamma), M, C, ptr(dx),
             ptr(dres),
             ptr(dgamma), ptr(dbeta), 0, ptr(work), None, None, None, None, stream())
        if ctx.has_res and not ctx.relu:
            dres = dout
        return dx, dgamma, dbeta, dres, None, None, None, None, None, None


def batch_norm(x, gamma, beta, rmean, rvar, training=True, momentum=0.99, eps=1e-3, relu=False, residual=None):
    """Channels-last FusedBatchNorm (+ optional residual add and ReLU)."""
    if on_gpu(x) and x.shape[-1] % 8 == 0:
        return _BNFn.apply(x.to(BF16), gamma, beta, residual, rmean, rvar, bool(relu), float(momentum), float(eps),
                           bool(training))
    y = batch_norm_ref(x, gamma, beta, rmean, rvar, momentum, eps, training)
    if residual is not None:
        y = y + residual.float()
    y = torch.relu(y) if relu else y
    return y.to(x.dtype) if x.is_floating_point() else y


class _LNFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, gamma, beta, eps, link=None):
        # link: ops.conv.ResidualGradLink on which the residual add of the same input parks its gradient; the
        # backward adds it in its store pass (pre-LN blocks: x feeds LN and the residual connection)
        ctx.link = link
        pend = take_pending(x)  # x = x0 + dropout(f) still to be formed (ops.add_dropout(..., into_ln=True))
        x = x.contiguous()
        D = x.shape[-1]
        M = x.numel() // D
        y = torch.empty_like(x)
        mean = torch.empty(M, dtype=F32, device=x.device)
        rstd = torch.empty(M, dtype=F32, device=x.device)
        if pend is not None:
            call("dtf_add_dropout_layernorm_fwd", ptr(pend.x), ptr(pend.f), ptr(x), ptr(gamma), ptr(beta), ptr(y),
                 ptr(mean), ptr(rstd), M, D, float(eps), float(pend.keep), int(pend.seed), pend.ctr, stream())
        else:
            call("dtf_layernorm_fwd", ptr(x), ptr(gamma), ptr(beta), ptr(y), ptr(mean), ptr(rstd), M, D, float(eps),
                 stream())
        ctx.save_for_backward(x, gamma, mean, rstd)
        ctx.ln_params = (gamma, beta)
        ctx.dsrc = getattr(x, "_dtf_dropsrc", None)  # x = x0 + dropout(f): apply that dropout's backward too
        return y

    @staticmethod
    def backward(ctx, dy):
        x, gamma, mean, rstd = ctx.saved_tensors
        D = x.shape[-1]
        M = x.numel() // D
        dy = dy.to(BF16).contiguous()
        dx = torch.empty_like(x)
        ws = workspace(x.device)
        res = ctx.link.take()[0] if ctx.link is not None else None
        ctx.link = None
        if res is not None:
            res = res.to(BF16).contiguous()
        g_p, b_p = ctx.ln_params
        tg, tb = direct_grad(g_p), direct_grad(b_p)
        if tg is not None and tb is not None and tb.data_ptr() == tg.data_ptr() + 4 * D and SIDE_STREAM_ON:
            # gamma and beta are adjacent in the arena: dx here, and the [dgamma | dbeta] partial rows reduced into
            # their gradients on the weight-gradient side stream — the reduction launches leave the dgrad chain,
            # where they waited for CUs held by side-stream GEMM blocks
            part = torch.empty(1024 * 2 * D, dtype=F32, device=x.device)
            rows = IntOut()
            src, ctx.dsrc = ctx.dsrc, None
            df = torch.empty_like(dx) if src is not None else None
            call("dtf_layernorm_bwd_part", ptr(dy), ptr(x), ptr(gamma), ptr(mean), ptr(rstd), ptr(dx), ptr(part),
                 part.numel(), M, D, ptr(res), rows.addr, ptr(df), float(src.keep) if src else 1.0,
                 int(src.seed) if src else 0, src.ctr if src else None, stream())
            if src is not None:
                src.provide(dx, df)
            with fork_side(x.device, part):
                call("dtf_sum_rows", ptr(part), 2 * D, rows.value, 2 * D, ptr(tg), 1, stream())
            return dx, None, None, None, None
        if tg is not None and tb is not None and tb.data_ptr() == tg.data_ptr() + 4 * D:
            # gamma and beta are adjacent in the arena: accumulate [dgamma | dbeta] into their gradients
            call("dtf_layernorm_bwd2", ptr(dy), ptr(x), ptr(gamma), ptr(mean), ptr(rstd), ptr(dx), ptr(tg), ptr(ws),
                 ws.numel(), M, D, 1, ptr(res), stream())
            return dx, None, None, None, None
        dgb = torch.empty(2 * D, dtype=F32, device=x.device)
        call("dtf_layernorm_bwd2", ptr(dy), ptr(x), ptr(gamma), ptr(mean), ptr(rstd), ptr(dx), ptr(dgb), ptr(ws),
             ws.numel(), M, D, 0, ptr(res), stream())
        return dx, dgb[:D], dgb[D:], None, None


def layer_norm(x, gamma, beta, eps=1e-5, link=None):
    """link: a ResidualGradLink shared with the residual add of the same input (ops.add_dropout(..., link=)):
    that add parks its gradient of x and this backward returns the sum (no autograd add kernel)."""
    if on_gpu(x) and x.shape[-1] % 8 == 0 and x.dtype == BF16:
        return _LNFn.apply(x, gamma, beta, float(eps), link)
    pend = take_pending(x)
    if pend is not None:  # (an input this LayerNorm cannot fuse: form the sum first)
        pend.resolve(x)
    if on_gpu(x) and x.shape[-1] % 8 == 0:
        return _LNFn.apply(x.to(BF16), gamma, beta, float(eps), link)
    return torch.nn.functional.layer_norm(x.float(), (x.shape[-1],), gamma, beta, eps).to(
        x.dtype if x.is_floating_point() else torch.float32)
