"""Pooling, activations, dropout, embeddings, softmax / cross-entropy ops
(csrc/kernels/pool.hip, elementwise.hip) with CPU references."""
from __future__ import annotations

import torch

from ._util import BF16, F32, call, direct_grad, on_gpu, ptr, rng_counter, stream, workspace
from .conv import out_size


# ------------------------------------------------------------------ pooling
class _MaxPoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k, s, p):
        x = x.contiguous()
        N, H, W, C = x.shape
        P, Q = out_size(H, k[0], s[0], p[0]), out_size(W, k[1], s[1], p[1])
        y = torch.empty((N, P, Q, C), dtype=BF16, device=x.device)
        arg = torch.empty((N, P, Q, C), dtype=torch.uint8, device=x.device)
        call("dtf_maxpool_fwd", ptr(x), ptr(y), ptr(arg), N, H, W, C, P, Q, k[0], k[1], s[0], s[1], p[0], p[1],
             stream())
        ctx.save_for_backward(arg)
        ctx.geo = (N, H, W, C, P, Q, k, s, p)
        return y

    @staticmethod
    def backward(ctx, dy):
        (arg,) = ctx.saved_tensors
        N, H, W, C, P, Q, k, s, p = ctx.geo
        dy = dy.to(BF16).contiguous()
        dx = torch.empty((N, H, W, C), dtype=BF16, device=dy.device)
        call("dtf_maxpool_bwd", ptr(dy), ptr(arg), ptr(dx), N, H, W, C, P, Q, k[0], k[1], s[0], s[1], p[0], p[1],
             stream())
        return dx, None, None, None


def max_pool2d(x, ksize=(3, 3), strides=(2, 2), pad=(1, 1)):
    ksize, strides, pad = tuple(ksize), tuple(strides), tuple(pad)
    if on_gpu(x) and x.shape[-1] % 8 == 0:
        return _MaxPoolFn.apply(x.to(BF16), ksize, strides, pad)
    y = torch.nn.functional.max_pool2d(x.permute(0, 3, 1, 2), ksize, strides, pad)
    return y.permute(0, 2, 3, 1)


class _GAPFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        x = x.contiguous()
        N, H, W, C = x.shape
        y = torch.empty((N, C), dtype=BF16, device=x.device)
        call("dtf_gap_fwd", ptr(x), ptr(y), N, H * W, C, 0, stream())
        ctx.geo = (N, H, W, C)
        return y

    @staticmethod
    def backward(ctx, dy):
        N, H, W, C = ctx.geo
        dy = dy.contiguous()
        dx = torch.empty((N, H, W, C), dtype=BF16, device=dy.device)
        call("dtf_gap_bwd", ptr(dy), int(dy.dtype == F32), ptr(dx), N, H * W, C, stream())
        return dx


def global_avg_pool(x):
    if on_gpu(x) and x.shape[-1] % 8 == 0:
        return _GAPFn.apply(x.to(BF16))
    return x.mean(dim=(1, 2))


# ------------------------------------------------------------------ activations
class _ActFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, act):
        x = x.contiguous()
        y = torch.empty_like(x)
        call("dtf_act", ptr(x), None, ptr(y), x.numel(), act, 0, stream())
        ctx.save_for_backward(x)
        ctx.act = act
        return y

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        dy = dy.to(BF16).contiguous()
        dx = torch.empty_like(x)
        call("dtf_act", ptr(x), ptr(dy), ptr(dx), x.numel(), ctx.act, 1, stream())
        return dx, None


def relu(x):
    if on_gpu(x) and x.dtype == BF16 and x.numel() % 8 == 0:
        return _ActFn.apply(x, 1)
    return torch.relu(x)


def gelu(x):
    if on_gpu(x) and x.dtype == BF16 and x.numel() % 8 == 0:
        return _ActFn.apply(x, 2)
    return torch.nn.functional.gelu(x, approximate="tanh")


class _DropoutFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, keep, seed, ctr):
        x = x.contiguous()
        y = torch.empty_like(x)
        call("dtf_dropout", ptr(x), ptr(y), x.numel(), float(keep), int(seed), ctr, stream())
        ctx.keep, ctx.seed, ctx.ctr = keep, seed, ctr
        return y

    @staticmethod
    def backward(ctx, dy):
        dy = dy.to(BF16).contiguous()
        dx = torch.empty_like(dy)
        call("dtf_dropout", ptr(dy), ptr(dx), dy.numel(), float(ctx.keep), int(ctx.seed), ctx.ctr, stream())
        return dx, None, None, None


_seed_counter = [0x5EED]


def _auto_seed(seed, device):
    """(host seed, device step-counter pointer or None): explicit seeds are stateless, automatic ones follow
    the per-step device counter (see _util.rng_counter)."""
    if seed is not None:
        return seed & 0xFFFFFFFFFFFFFFFF, None
    _seed_counter[0] += 1
    return (_seed_counter[0] * 0x9E3779B1) & 0xFFFFFFFFFFFFFFFF, rng_counter(device)


def dropout(x, rate, training=True, seed=None):
    if not training or rate <= 0.0:
        return x
    keep = 1.0 - rate
    if on_gpu(x) and x.dtype == BF16 and x.numel() % 8 == 0:
        s, ctr = _auto_seed(seed, x.device)
        return _DropoutFn.apply(x, keep, s, ctr)
    return torch.nn.functional.dropout(x, rate, True)


_FUSE_ADD_DROPOUT = True


class DropSource:
    """What a LayerNorm consuming an add_dropout output needs to apply that dropout's backward in its own store pass
    (norm.hip ln_bwd_kernel dfo): the mask parameters; the LayerNorm backward leaves df here and add_dropout's backward
    takes it when the gradient it receives is exactly the tensor that LayerNorm backward wrote (its only consumer, or
    the residual joined inside the LayerNorm backward) — otherwise it runs its own dropout pass."""
    __slots__ = ("keep", "seed", "ctr", "df", "dx", "ver", "__weakref__")

    def __init__(self, keep, seed, ctr):
        self.keep, self.seed, self.ctr = keep, seed, ctr
        self.df = self.dx = self.ver = None

    def provide(self, dx, df):
        # hold dx itself (not only its address): a freed dx whose address a later gradient reuses can never match
        self.df, self.dx, self.ver = df, dx, dx._version

    def take(self, dy):
        df, dx, ver = self.df, self.dx, self.ver
        self.df = self.dx = self.ver = None
        return df if (df is not None and same_unmodified(dy, dx, ver)) else None


def same_unmodified(t, src, ver):
    """t is (a view of) the very buffer `src` that a fused backward wrote, with no in-place write since (the version
    counter is shared by all views of a storage: an autograd accumulation into it bumps it)."""
    return (src is not None and t.data_ptr() == src.data_ptr() and t.shape == src.shape and t.is_contiguous()
            and src._version == ver and t._version == ver)


class _AddDropoutFn(torch.autograd.Function):
    """y = x + dropout(f): one pass forward; backward dx = dy, df = dropout(dy) with the same mask (or df from the
    consuming LayerNorm's backward, DropSource)."""

    @staticmethod
    def forward(ctx, x, f, keep, seed, ctr, link, defer=False):
        x, f = x.contiguous(), f.contiguous()
        y = torch.empty_like(x)
        if defer:
            # formed by the LayerNorm this output feeds (ops.norm.layer_norm resolves it: one fused pass)
            y._dtf_pending = PendingAddDropout(x, f, keep, seed, ctr)
        else:
            call("dtf_add_dropout", ptr(x), ptr(f), ptr(y), x.numel(), float(keep), int(seed), ctr, stream())
        ctx.keep, ctx.seed, ctx.ctr, ctx.link = keep, seed, ctr, link
        ctx.src = DropSource(keep, seed, ctr) if _FUSE_LN_DROPOUT_BWD else None
        if ctx.src is not None:
            y._dtf_dropsrc = ctx.src
        return y

    @staticmethod
    def backward(ctx, dy):
        dy = dy.to(BF16).contiguous()
        df = ctx.src.take(dy) if ctx.src is not None else None
        ctx.src = None
        if df is None:
            df = torch.empty_like(dy)
            call("dtf_dropout", ptr(dy), ptr(df), dy.numel(), float(ctx.keep), int(ctx.seed), ctx.ctr, stream())
        dx = ctx.link.park(dy) if ctx.link is not None else dy  # None: the branch's first GEMM adds it
        ctx.link = None
        return dx, df, None, None, None, None, None


class PendingAddDropout:
    """An add_dropout output whose values are formed by the LayerNorm that consumes it (the model promises that the
    LayerNorm is its first reader: models.transformer passes defer=True only there). resolve() forms them with the
    plain add kernel when that LayerNorm cannot fuse."""
    __slots__ = ("x", "f", "keep", "seed", "ctr")

    def __init__(self, x, f, keep, seed, ctr):
        self.x, self.f, self.keep, self.seed, self.ctr = x, f, keep, seed, ctr

    def resolve(self, y):
        call("dtf_add_dropout", ptr(self.x), ptr(self.f), ptr(y), y.numel(), float(self.keep), int(self.seed), self.ctr,
             stream())


def take_pending(y):
    """The PendingAddDropout of y (cleared), or None."""
    p = getattr(y, "_dtf_pending", None)
    if p is not None:
        y._dtf_pending = None
    return p


# A LayerNorm whose input is an add_dropout output applies the dropout's backward in its own store pass (module
# switch for tests: tests/test_model_training_gpu.py compares both).
_FUSE_LN_DROPOUT_BWD = True


# add_dropout(..., into_ln=True) leaves its sum to the LayerNorm it feeds (one fused pass forward)
_FUSE_ADD_LN = True


def add_dropout(x, f, rate, training=True, seed=None, link=None, into_ln=False):
    """Residual connection around a dropped-out branch: x + dropout(f, rate) (fused on GPU). link: a
    ResidualGradLink shared with the branch's first Dense layer (ops.dense(..., link=)): the residual gradient
    of x is then added inside that layer's data-gradient GEMM instead of by autograd. into_ln: the caller feeds the
    result to ops.layer_norm before anything else reads it; the sum is then formed in the LayerNorm's pass."""
    if not training or rate <= 0.0:
        return add(x, f)
    if _FUSE_ADD_DROPOUT and on_gpu(x) and x.dtype == BF16 and f.dtype == BF16 and x.shape == f.shape \
            and x.numel() % 8 == 0:
        s, ctr = _auto_seed(seed, x.device)
        defer = bool(into_ln and _FUSE_ADD_LN and x.shape[-1] % 8 == 0 and x.shape[-1] <= 2048)
        return _AddDropoutFn.apply(x, f, 1.0 - rate, s, ctr, link, defer)
    return add(x, dropout(f, rate, training, seed))


def add(a, b):
    if on_gpu(a) and a.dtype == BF16 and b.dtype == BF16 and a.numel() % 8 == 0 and a.shape == b.shape:
        return _AddFn.apply(a, b)
    return a + b


class _AddFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, b):
        a, b = a.contiguous(), b.contiguous()
        y = torch.empty_like(a)
        call("dtf_add_bf16", ptr(a), ptr(b), ptr(y), a.numel(), 1.0, 1.0, stream())
        return y

    @staticmethod
    def backward(ctx, dy):
        return dy, dy


# ------------------------------------------------------------------ sort / indexed rows
def sort_keys(keys, key_bits=None):
    """(sorted keys, permutation) of a 1-D int64 tensor of non-negative keys < 2^key_bits — a stable sort: equal keys
    keep their input order (csrc/kernels/sort.hip radix sort on GPU; torch.sort(stable=True) on the CPU)."""
    keys = keys.reshape(-1).long().contiguous()
    if not on_gpu(keys):
        return torch.sort(keys, stable=True)
    n = keys.numel()
    if key_bits is None:
        raise ValueError("sort_keys on the GPU needs key_bits (the key range), read from no device value")
    sk = torch.empty_like(keys)
    perm = torch.empty_like(keys)
    ws_bytes = 2 * n * 8 + 256 * ((n + 1023) // 1024) * 4 + 64
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=keys.device)
    call("dtf_sort_keys", ptr(keys), n, int(key_bits), ptr(sk), ptr(perm), ptr(ws), ws_bytes, stream())
    return sk, perm


def _bits(n):
    return max(1, int(n - 1).bit_length())


class _GatherRowsFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, src, idx):
        src, idx = src.contiguous(), idx.reshape(-1).long().contiguous()
        R, D = src.shape
        out = torch.empty((idx.numel(), D), dtype=src.dtype, device=src.device)
        call("dtf_gather_rows", ptr(src), ptr(idx), ptr(out), idx.numel(), D, stream())
        ctx.save_for_backward(idx)
        ctx.R = R
        return out

    @staticmethod
    def backward(ctx, dy):
        idx, = ctx.saved_tensors
        dy = dy.to(BF16).contiguous()
        sidx, perm = sort_keys(idx, _bits(ctx.R))
        ds = torch.empty((ctx.R, dy.shape[1]), dtype=BF16, device=dy.device)
        call("dtf_gather_rows_bwd", ptr(dy), ptr(sidx), ptr(perm), idx.numel(), ptr(ds), ctx.R, dy.shape[1], stream())
        return ds, None


def gather_rows(src, idx):
    """src[idx] for a 2-D bf16 src and 1-D row indices (the masked-LM gather); its gradient sums the rows gathered
    more than once in a fixed order and writes zeros elsewhere (deterministic, no fill pass, no atomics)."""
    if on_gpu(src) and src.dtype == BF16 and src.dim() == 2 and src.shape[1] % 8 == 0:
        return _GatherRowsFn.apply(src, idx)
    return src.index_select(0, idx.reshape(-1).long())


# ------------------------------------------------------------------ embeddings
class _EmbedFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, ids, table, pos_table, type_ids, type_table, seq_len):
        ids = ids.contiguous().long()
        T = ids.numel()
        D = table.shape[1]
        from ._util import bf16_shadow
        t16 = bf16_shadow(table)
        p16 = bf16_shadow(pos_table) if pos_table is not None else None
        y16 = bf16_shadow(type_table) if type_table is not None else None
        tid = type_ids.contiguous().long() if type_ids is not None else None
        out = torch.empty((T, D), dtype=BF16, device=ids.device)
        call("dtf_embed_fwd", ptr(t16), ptr(ids), ptr(p16), None, ptr(y16), ptr(tid), ptr(out), T, D, int(seq_len),
             stream())
        ctx.save_for_backward(ids, tid)
        ctx.tables = (table, pos_table, type_table)
        ctx.shapes = (table.shape, None if pos_table is None else pos_table.shape,
                      None if type_table is None else type_table.shape, seq_len)
        return out.reshape(*ids.shape, D)

    @staticmethod
    def backward(ctx, dy):
        ids, tid = ctx.saved_tensors
        tshape, pshape, yshape, seq_len = ctx.shapes
        dy = dy.to(BF16).contiguous()
        T = ids.numel()
        D = tshape[1]
        ws = workspace(dy.device)
        tables = ctx.tables
        # inside Model.train_step the kernels accumulate straight into the arena gradients (no zero-filled
        # temporaries, no AccumulateGrad adds); the returned gradient is then None
        direct = [direct_grad(t) for t in tables]
        # word table: sort the ids once, then one deterministic segment-sum per distinct id (no atomics)
        dt = direct[0] if direct[0] is not None else torch.zeros(tshape, dtype=F32, device=dy.device)
        sid, perm = sort_keys(ids, _bits(tshape[0]))
        call("dtf_embed_bwd_sorted", ptr(dy), ptr(sid), ptr(perm), ptr(dt), T, D, stream())
        dp = dy_ = None
        if pshape is not None:  # positions: dp[s] = sum over the batch of dy[b, s]  (a column sum)
            dp = direct[1] if direct[1] is not None else torch.zeros(pshape, dtype=F32, device=dy.device)
            S = int(seq_len)
            call("dtf_colsum", ptr(dy), T // S, S * D, ptr(dp), int(direct[1] is not None), ptr(ws), ws.numel(),
                 stream())
        if yshape is not None:
            acc = int(direct[2] is not None)
            dy_ = direct[2] if acc else torch.zeros(yshape, dtype=F32, device=dy.device)
            if tid is not None and yshape[0] <= 16 and D <= 2048:
                call("dtf_embed_bwd_small", ptr(dy), ptr(tid), ptr(dy_), T, D, yshape[0], acc, ptr(ws), ws.numel(),
                     stream())
            elif tid is not None:
                sid2, perm2 = sort_keys(tid, _bits(yshape[0]))
                call("dtf_embed_bwd_sorted", ptr(dy), ptr(sid2), ptr(perm2), ptr(dy_), T, D, stream())
            else:  # no type ids: every token uses row 0
                call("dtf_colsum", ptr(dy), T, D, ptr(dy_), acc, ptr(ws), ws.numel(), stream())
        dt = None if direct[0] is not None else dt
        dp = None if direct[1] is not None else dp
        dy_ = None if direct[2] is not None else dy_
        return None, dt, dp, None, dy_, None


def embedding(ids, table, pos_table=None, type_ids=None, type_table=None):
    """out[..., :] = table[ids] (+ pos_table[position]) (+ type_table[type_ids]); positions = last axis index."""
    seq_len = ids.shape[-1]
    if on_gpu(ids) and table.shape[1] % 8 == 0:
        return _EmbedFn.apply(ids, table, pos_table, type_ids, type_table, seq_len)
    out = table[ids.long()]
    if pos_table is not None:
        out = out + pos_table[:seq_len]
    if type_table is not None:
        out = out + (type_table[type_ids.long()] if type_ids is not None else type_table[0])
    return out


# ------------------------------------------------------------------ softmax / losses
class _SoftmaxCEFn(torch.autograd.Function):
    """Forward: one online pass per row (loss, logsumexp); backward: ONE pass writing
    (softmax - target) * dloss[row] — the logits are read twice and the gradient written once in total."""

    @staticmethod
    def forward(ctx, logits, labels, smooth):
        logits = logits.contiguous()
        labels = labels.contiguous().long()
        V = logits.shape[-1]
        rows = logits.numel() // V
        loss = torch.empty(rows, dtype=F32, device=logits.device)
        lse = torch.empty(rows, dtype=F32, device=logits.device)
        call("dtf_softmax_ce_fwd", ptr(logits), int(logits.dtype == F32), ptr(labels), ptr(loss), ptr(lse), rows, V,
             float(smooth), stream())
        ctx.save_for_backward(logits, labels, lse)
        ctx.smooth = float(smooth)
        return loss.reshape(logits.shape[:-1])

    @staticmethod
    def backward(ctx, dloss):
        logits, labels, lse = ctx.saved_tensors
        V = logits.shape[-1]
        rows = logits.numel() // V
        g = dloss.reshape(-1).to(F32).expand(rows).contiguous()
        dl = torch.empty_like(logits)
        call("dtf_softmax_ce_bwd", ptr(logits), int(logits.dtype == F32), ptr(labels), ptr(lse), ptr(g), ptr(dl),
             rows, V, ctx.smooth, stream())
        return dl, None, None


def sparse_softmax_cross_entropy(logits, labels, label_smoothing=0.0):
    """Per-example loss of tf.nn.sparse_softmax_cross_entropy_with_logits (fused fwd+grad kernel)."""
    if on_gpu(logits):
        return _SoftmaxCEFn.apply(logits, labels, float(label_smoothing))
    return torch.nn.functional.cross_entropy(logits.float().reshape(-1, logits.shape[-1]), labels.reshape(-1).long(),
                                             reduction="none", label_smoothing=label_smoothing,
                                             ignore_index=-100).reshape(labels.shape)


class _SoftmaxFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, scale, causal, add_mask):
        x = x.contiguous()
        Sq, Sk = x.shape[-2], x.shape[-1]
        rows = x.numel() // Sk
        y = torch.empty_like(x)
        call("dtf_softmax_fwd", ptr(x), ptr(y), rows, Sq, Sk, float(scale), int(causal), ptr(add_mask), stream())
        ctx.save_for_backward(y)
        ctx.scale = scale
        return y

    @staticmethod
    def backward(ctx, dy):
        (y,) = ctx.saved_tensors
        dy = dy.to(BF16).contiguous()
        Sk = y.shape[-1]
        dx = torch.empty_like(y)
        call("dtf_softmax_bwd", ptr(y), ptr(dy), ptr(dx), y.numel() // Sk, Sk, float(ctx.scale), stream())
        return dx, None, None, None


def softmax(x, scale=1.0, causal=False, add_mask=None):
    """Row softmax(scale*x + mask) over the last axis.

    add_mask: optional f32 additive mask of shape [prod(x.shape[:-2]), Sk] (one row per score matrix)."""
    if on_gpu(x) and x.dtype == BF16:
        return _SoftmaxFn.apply(x, float(scale), bool(causal), add_mask)
    z = x.float() * scale
    if causal:
        Sq, Sk = z.shape[-2], z.shape[-1]
        m = torch.ones(Sq, Sk, dtype=torch.bool, device=z.device).tril(Sk - Sq)
        z = z.masked_fill(~m, float("-inf"))
    if add_mask is not None:
        z = z + add_mask.reshape(*z.shape[:-2], 1, z.shape[-1])
    return torch.softmax(z, dim=-1).to(x.dtype)
