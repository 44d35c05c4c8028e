"""BERT-base (post-LN encoder, MLM + NSP heads) and GPT-2 (pre-LN causal decoder, tied LM head).

BASELINE.json configs: "BERT-base seq=512 MultiWorkerMirroredStrategy" and "GPT-2-medium fp8 weights
MirroredStrategy". Dense layers run on the MFMA GEMM with fused bias/GELU epilogues; LayerNorm,
softmax, embeddings and the vocab cross-entropy on their HIP kernels. ``fp8=True`` runs the
projection GEMMs of the transformer blocks with OCP e4m3 operands (CDNA4 fp8 MFMA, per-tensor
delayed scaling — ops.fp8).
"""
from __future__ import annotations

import math

import torch

from .. import ops
from ..ops import mha as attn_ops
from ..keras import layers as KL
from ..keras.models import Model
from ..ops.conv import ResidualGradLink

# post-LN blocks (BERT): the residual gradient of a sublayer's input is added by the sublayer's first projection's
# data-gradient GEMM in its store pass, in place in the parked buffer (no clone, no add kernel): BERT-base 19.60 ->
# 19.40 ms/step, bitwise-equal losses
RES_LINK = True
# pre-LN blocks (GPT-2): the residual gradient is added in the LayerNorm backward's store pass (GPT-2-medium bf16
# 35.50 -> 35.35, fp8 34.84 -> 34.48 ms/step, bitwise-equal results)
LN_LINK = True


class _Proj(KL.Layer):
    """Dense [units, in] with optional fp8 forward."""

    def __init__(self, units, activation=None, fp8=False, init_std=0.02, single_consumer=False, **kw):
        super().__init__(**kw)
        self.units, self.activation, self.fp8, self.init_std = units, activation, fp8, init_std
        # the output feeds exactly one _Proj (FFN1 -> FFN2): its activation backward may be fused downstream
        self.single_consumer = single_consumer

    def build(self, input_shape):
        from ..keras.initializers import TruncatedNormal
        self.kernel = self.add_weight("kernel", (self.units, input_shape[-1]), TruncatedNormal(0.0, self.init_std))
        self.bias = self.add_weight("bias", (self.units,), "zeros")
        self.built = True

    def call(self, x, training=None, link=None):
        if self.fp8 and x.is_cuda:
            from ..ops.fp8 import dense_fp8
            return dense_fp8(x, self.kernel, self.bias, self.activation, self, getattr(self, "_fp8_next", None))
        return ops.dense(x, self.kernel, self.bias, act=self.activation, link=link, tag_act=self.single_consumer)


class MultiHeadSelfAttention(KL.Layer):
    def __init__(self, hidden, heads, dropout=0.1, causal=False, fp8=False, **kw):
        super().__init__(**kw)
        self.heads, self.dropout, self.causal = heads, dropout, causal
        self.qkv = _Proj(3 * hidden, fp8=fp8)
        self.out = _Proj(hidden, fp8=fp8)

    def call(self, x, mask=None, training=None, link=None):
        o = attn_ops.attention_packed(self.qkv(x, link=link), self.heads, causal=self.causal, mask=mask,
                                      dropout=self.dropout, training=training)
        return self.out(o)


class BertLayer(KL.Layer):
    def __init__(self, hidden=768, heads=12, ffn=3072, dropout=0.1, **kw):
        super().__init__(**kw)
        self.att = MultiHeadSelfAttention(hidden, heads, dropout)
        self.ln1 = KL.LayerNormalization(epsilon=1e-12)
        self.ff1 = _Proj(ffn, activation="gelu", single_consumer=True)
        self.ff2 = _Proj(hidden)
        self.ln2 = KL.LayerNormalization(epsilon=1e-12)
        self.dropout = dropout

    def call(self, x, mask=None, training=None):
        # residual gradients of x join the data-gradient GEMM of the branch's first projection (ResidualGradLink)
        l1, l2 = (ResidualGradLink(), ResidualGradLink()) if (RES_LINK and training and x.is_cuda
                                                              and torch.is_grad_enabled()) else (None, None)
        a = self.att(x, mask, training=training, link=l1)
        # (into_ln: each residual sum is formed inside the LayerNorm pass that reads it first)
        x = self.ln1(ops.add_dropout(x, a, self.dropout, bool(training), link=l1, into_ln=True))
        f = self.ff2(self.ff1(x, link=l2))
        return self.ln2(ops.add_dropout(x, f, self.dropout, bool(training), link=l2, into_ln=True))


class BertModel(Model):
    """BERT encoder with MLM (tied decoder) and NSP heads. Inputs: ids, type_ids, attention mask."""

    def __init__(self, vocab=30522, hidden=768, layers=12, heads=12, ffn=3072, max_pos=512, type_vocab=2,
                 dropout=0.1, name="bert", **kw):
        super().__init__(name=name, **kw)
        self.cfg = dict(vocab=vocab, hidden=hidden, layers=layers, heads=heads, ffn=ffn, max_pos=max_pos)
        from ..keras.initializers import TruncatedNormal
        # vocab padded to a multiple of 64 (MFMA tiles); padded logits carry a -1e9 bias -> zero probability
        self.vocab, self.vocab_p = vocab, (vocab + 63) // 64 * 64
        self.word = self.add_weight("embeddings/word", (self.vocab_p, hidden), TruncatedNormal(0.0, 0.02))
        self.pos = self.add_weight("embeddings/position", (max_pos, hidden), TruncatedNormal(0.0, 0.02))
        self.typ = self.add_weight("embeddings/type", (type_vocab, hidden), TruncatedNormal(0.0, 0.02))
        self.emb_ln = KL.LayerNormalization(epsilon=1e-12)
        self.blocks = [BertLayer(hidden, heads, ffn, dropout) for _ in range(layers)]
        self.mlm_dense = _Proj(hidden, activation="gelu")
        self.mlm_ln = KL.LayerNormalization(epsilon=1e-12)
        self.mlm_bias = self.add_weight("mlm/bias", (self.vocab_p,), "zeros")
        with torch.no_grad():
            self.mlm_bias[vocab:] = -1e9
        self.pool = _Proj(hidden)
        self.nsp = _Proj(2)
        self.dropout = dropout
        self.built = True

    def encode(self, ids, type_ids=None, attn_mask=None, training=None):
        x = ops.embedding(ids, self.word, self.pos, type_ids, self.typ)
        x = ops.dropout(self.emb_ln(x), self.dropout, training=bool(training))
        mask = None
        if attn_mask is not None:
            mask = (1.0 - attn_mask.float()) * -10000.0
        for b in self.blocks:
            x = b(x, mask, training=training)
        return x

    def mlm_logits(self, h):
        t = self.mlm_ln(self.mlm_dense(h))
        return ops.dense(t, self.word, self.mlm_bias)

    def call(self, inputs, training=None):
        if isinstance(inputs, dict):
            ids, tids, am = inputs["input_ids"], inputs.get("token_type_ids"), inputs.get("attention_mask")
            mpos = inputs.get("masked_positions")
        else:
            ids, tids, am, mpos = inputs, None, None, None
        h = self.encode(ids, tids, am, training=training)
        if mpos is not None:  # gather the masked positions only (BERT pretraining)
            B, S, Hd = h.shape
            idx = (mpos + torch.arange(B, device=mpos.device)[:, None] * S).reshape(-1)
            h = ops.gather_rows(h.reshape(B * S, Hd), idx).reshape(B, -1, Hd)
        return self.mlm_logits(h)

    def nsp_logits(self, h):
        return self.nsp(torch.tanh(self.pool(h[:, 0]).float()).to(h.dtype))


class GPT2Block(KL.Layer):
    def __init__(self, hidden, heads, dropout=0.1, fp8=False, **kw):
        super().__init__(**kw)
        self.ln1 = KL.LayerNormalization(epsilon=1e-5)
        self.att = MultiHeadSelfAttention(hidden, heads, dropout, causal=True, fp8=fp8)
        self.ln2 = KL.LayerNormalization(epsilon=1e-5)
        self.fc = _Proj(4 * hidden, activation="gelu", fp8=fp8, single_consumer=True)
        self.proj = _Proj(hidden, fp8=fp8)
        if fp8:  # FFN1's output feeds only FFN2: fp8 operands from FFN1's epilogue (ops.fp8 _FUSE); untracked
            object.__setattr__(self.fc, "_fp8_next", self.proj)
        self.dropout = dropout
        object.__setattr__(self, "out_into_ln", False)  # set by GPT2: the output's first reader is a LayerNorm

    def call(self, x, training=None):
        # the residual gradient of each half-block's input joins its LayerNorm's backward (ResidualGradLink)
        l1, l2 = (ResidualGradLink(), ResidualGradLink()) if (LN_LINK and training and x.is_cuda
                                                              and torch.is_grad_enabled()) else (None, None)
        # (into_ln: the residual sum is formed inside the LayerNorm pass that reads it first — ln2 here; the block
        # output only when the owning GPT2 feeds it to the next block's ln1 or ln_f, out_into_ln)
        x = ops.add_dropout(x, self.att(self.ln1(x, link=l1), training=training), self.dropout, bool(training),
                            link=l1, into_ln=True)
        return ops.add_dropout(x, self.proj(self.fc(self.ln2(x, link=l2))), self.dropout, bool(training), link=l2,
                               into_ln=self.out_into_ln)


class GPT2(Model):
    def __init__(self, vocab=50257, ctx=1024, hidden=1024, layers=24, heads=16, dropout=0.1, fp8=False,
                 name="gpt2", **kw):
        super().__init__(name=name, **kw)
        # per-bucket optimizer update during backward (parallel.strategy): round 4, with the plain GEMMs on hipBLASLt,
        # it pays for bf16 (256.0k / 255.6k vs 251.2k / 251.3k tok/s) and no longer for fp8 (248.6k / 258.2k vs
        # 256.9k / 256.5k, with 3-6 ms more host issue time); round 3 had measured the opposite (fp8 +2%, bf16 -1%)
        self.overlap_update = not fp8
        self.cfg = dict(vocab=vocab, ctx=ctx, hidden=hidden, layers=layers, heads=heads, fp8=fp8)
        from ..keras.initializers import TruncatedNormal
        # vocab padded to a multiple of 64 for the MFMA tiles (padded logits are masked out of the loss)
        self.vocab = vocab
        self.vocab_p = (vocab + 63) // 64 * 64
        self.wte = self.add_weight("wte", (self.vocab_p, hidden), TruncatedNormal(0.0, 0.02))
        self.wpe = self.add_weight("wpe", (ctx, hidden), TruncatedNormal(0.0, 0.01))
        self.blocks = [GPT2Block(hidden, heads, dropout, fp8) for _ in range(layers)]
        for b in self.blocks:  # each block output is read first by the next block's ln1 or by ln_f
            object.__setattr__(b, "out_into_ln", True)
        self.ln_f = KL.LayerNormalization(epsilon=1e-5)
        pad = torch.zeros(self.vocab_p)
        pad[vocab:] = -1e9  # padded vocab entries never receive probability mass
        self.pad_bias = self.add_weight("lm_pad_bias", (self.vocab_p,), "zeros", trainable=False)
        with torch.no_grad():
            self.pad_bias.copy_(pad.to(self.pad_bias.device))
        self.dropout = dropout
        self.built = True

    def call(self, ids, training=None):
        x = ops.dropout(ops.embedding(ids, self.wte, self.wpe), self.dropout, training=bool(training))
        for b in self.blocks:
            x = b(x, training=training)
        return ops.dense(self.ln_f(x), self.wte, self.pad_bias)  # tied LM head, logits over vocab_p


def bert_base(**kw):
    return BertModel(**kw)


def gpt2_medium(fp8=False, **kw):
    return GPT2(hidden=1024, layers=24, heads=16, fp8=fp8, **kw)


def gpt2_small(fp8=False, **kw):
    return GPT2(hidden=768, layers=12, heads=12, fp8=fp8, **kw)


def count_flops_per_token(cfg, seq):
    """Approximate training FLOPs/token (6N + attention) for throughput reporting."""
    h, L = cfg["hidden"], cfg["layers"]
    n = 12 * L * h * h
    return 6 * n + 12 * L * h * seq


del math
