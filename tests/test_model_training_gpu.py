"""Whole-model training on the HIP path against a CPU reference of the same model.

A reduced-width ResNet (the bench model's exact code path: s2d stem + fused BN/ReLU/max-pool, ConvBN bottlenecks
with fused BN statistics, residual-gradient links, weight gradients on the side stream, fused SGD-momentum arena
update) and a BERT-tiny (embedding, LayerNorm, fused attention, GELU FFN, tied MLM decoder, AdamW) each train 10
steps on the GPU through Model.train_step; the same model with the same initial weights and batches trains on the
CPU reference ops (f32, with the ResNet's conv/BN outputs rounded to bf16 where the GPU stores them, as in
tests/test_resnet_gpu.py). The loss trajectories and the final weights must agree within bf16 tolerances — a wrong
kernel, a missed gradient, a stale bf16 shadow or a broken optimizer update moves them far outside."""
import numpy as np
import pytest
import torch

from distributed_tensorflow_amd.keras import initializers, losses, optimizers

pytestmark = pytest.mark.gpu


def _train(model_fn, opt_fn, batches, device, patch=None):
    from distributed_tensorflow_amd import context
    out = []
    with context.device(device):  # (weights are built lazily by the first step: keep it in the scope)
        m = model_fn()
        m.compile(optimizer=opt_fn(), loss=losses.SparseCategoricalCrossentropy(from_logits=True))
        for x, y in batches:
            x = {k: v.to(device) for k, v in x.items()} if isinstance(x, dict) else x.to(device)
            out.append(float(m.train_step((x, y.to(device)))["loss"]))
    if device.type == "cuda":
        torch.cuda.synchronize()
    # by position: layer names carry per-process instance counters, the two models get different suffixes
    return out, {i: w.detach().float().cpu().numpy().copy() for i, w in enumerate(m.weights)}


def _rel(a, b):
    return float(np.linalg.norm(a - b) / (np.linalg.norm(b) + 1e-12))


def _one_step_update(dev, model_fn, x, y):
    """-gradient of every weight after one SGD(lr=1) step through Model.train_step (the whole training path)."""
    from distributed_tensorflow_amd import context
    with context.device(dev):
        m = model_fn()
        m.compile(optimizer=optimizers.SGD(1.0), loss=losses.SparseCategoricalCrossentropy(from_logits=True))
        with torch.no_grad():
            m(x.to(dev)[:1], training=False)
        before = [w.detach().float().cpu().clone() for w in m.weights]
        loss = float(m.train_step((x.to(dev), y.to(dev)))["loss"])
        return loss, [b - w.detach().float().cpu() for b, w in zip(before, m.weights)]


def _median_rel(a_list, b_list):
    return float(np.median([float((a - b).norm() / (b.norm() + 1e-12)) for a, b in zip(a_list, b_list)
                            if b.numel() > 1]))


def test_resnet_trains_like_cpu_reference(cuda, monkeypatch):
    """A random-init BN ResNet on random labels is badly conditioned: a 1e-3 input perturbation moves its
    gradients by ~50% (median over parameters) on the CPU reference itself (measured with
    tools/debug_model_vs_cpu.py). So the HIP path must (a) match the forward loss within 1%, (b) deviate from the
    bf16-emulating reference by clearly LESS than that intrinsic sensitivity, and (c) train: 10 SGD steps over
    two revisited batches lower the loss on the GPU as on the CPU."""
    from distributed_tensorflow_amd.models import ResNet
    g = torch.Generator().manual_seed(0)
    two = [(torch.randn(8, 3, 64, 64, generator=g), torch.randint(0, 10, (8,), generator=g)) for _ in range(2)]
    noise = 1e-3 * torch.randn(two[0][0].shape, generator=g)

    def model_fn():
        initializers.set_seed(11)
        return ResNet(26, num_classes=10, width=16)

    def opt_fn():
        return optimizers.SGD(0.02, momentum=0.9)

    lg, ug = _one_step_update(cuda, model_fn, *two[0])
    gl, _ = _train(model_fn, opt_fn, two * 5, cuda)
    import test_resnet_gpu as emu
    from distributed_tensorflow_amd import ops
    from distributed_tensorflow_amd.ops import conv as OC
    monkeypatch.setattr(ops, "conv_bn", emu._emu_conv_bn)  # the layers' entry point
    monkeypatch.setattr(OC, "conv_bn", emu._emu_conv_bn)   # the CPU stem (conv_bn_maxpool) calls it too
    cpu = torch.device("cpu")
    lc, uc = _one_step_update(cpu, model_fn, *two[0])
    _, uc2 = _one_step_update(cpu, model_fn, two[0][0] + noise, two[0][1])
    cl, _ = _train(model_fn, opt_fn, two * 5, cpu)
    assert abs(lg - lc) <= 0.01 * abs(lc), (lg, lc)
    err, sens = _median_rel(ug, uc), _median_rel(uc2, uc)
    assert err < 0.75 * sens, (err, sens)
    assert all(np.isfinite(gl))
    for ls in (gl, cl):  # the last visit of each batch scores below its first
        assert ls[-2] < ls[0] and ls[-1] < ls[1], (gl, cl)


def _frozen_bn_grads(dev, x, y, ref_weights=None):
    """Gradients of the cross-entropy through a reduced ResNet with its BatchNorms in inference mode (running
    statistics from 3 training-mode forwards of the same batch on the CPU, copied into the device model)."""
    from distributed_tensorflow_amd import context
    from distributed_tensorflow_amd.models import ResNet
    with context.device(dev):
        initializers.set_seed(11)
        m = ResNet(26, num_classes=10, width=16)
        with torch.no_grad():
            if ref_weights is None:
                for _ in range(3):
                    m(x.to(dev), training=True)
            else:
                m(x.to(dev)[:1], training=False)
                for w, r in zip(m.weights, ref_weights):
                    w.data.copy_(r.to(dev))
        logits = m(x.to(dev), training=False).float()
        loss = torch.nn.functional.cross_entropy(logits, y.to(dev))
        grads = torch.autograd.grad(loss, m.trainable_weights)
        return float(loss), [g.detach().float().cpu() for g in grads], [w.detach().float().cpu() for w in m.weights]


def test_resnet_frozen_bn_gradients_match_cpu_reference(cuda, monkeypatch):
    """Well-conditioned whole-model gradient check. With batch-statistics BN the gradient of a
    random-init ResNet is chaotic: the f32 CPU reference itself moves by a median 23% per parameter under a 1e-3
    input perturbation, and bf16 rounding alone by 33-49% (profiles/r3_resnet_grad_calibration.txt), so no bf16
    implementation can match it per layer. With the BatchNorms frozen (inference mode, running statistics: Keras
    fine-tuning semantics) the same network is well conditioned (f32: 3.3% at 1e-3), and every parameter's
    gradient through the HIP path (s2d stem conv, fused ConvBN forward, frozen-BN backward, conv dgrad/wgrad on the
    MFMA kernels, residual joins, max-pool, global pool, Dense) must match the bf16-emulating CPU reference at a
    small median relative error, on fixed learnable (teacher) labels."""
    g = torch.Generator().manual_seed(0)
    x = torch.randn(8, 3, 64, 64, generator=g)
    t = torch.randn(3 * 16, 10, generator=torch.Generator().manual_seed(99))
    y = (torch.nn.functional.adaptive_avg_pool2d(x, 4).flatten(1) @ t).argmax(1)
    import test_resnet_gpu as emu
    from distributed_tensorflow_amd import ops
    from distributed_tensorflow_amd.ops import conv as OC
    gpu_ops = (ops.conv_bn, OC.conv_bn)
    monkeypatch.setattr(ops, "conv_bn", emu._emu_conv_bn)
    monkeypatch.setattr(OC, "conv_bn", emu._emu_conv_bn)
    cpu = torch.device("cpu")
    lc, gc, wc = _frozen_bn_grads(cpu, x, y)
    monkeypatch.setattr(ops, "conv_bn", gpu_ops[0])
    monkeypatch.setattr(OC, "conv_bn", gpu_ops[1])
    lg, gg, _ = _frozen_bn_grads(cuda, x, y, ref_weights=wc)
    assert abs(lg - lc) <= 0.01 * abs(lc), (lg, lc)
    rel = [float((a - b).norm() / (b.norm() + 1e-12)) for a, b in zip(gg, gc) if b.numel() > 1]
    med = float(np.median(rel))
    assert all(np.isfinite(rel)) and med <= 0.05, (med, sorted(rel)[-5:])


def test_bert_tiny_trains_like_cpu_reference(cuda):
    from distributed_tensorflow_amd.models.transformer import BertModel
    g = torch.Generator().manual_seed(1)
    B, S, P, V = 4, 64, 8, 1000
    batches = []
    for _ in range(2):  # revisited 5x each: the MLM loss must go down
        ids = torch.randint(0, V, (B, S), generator=g)
        mpos = torch.stack([torch.randperm(S, generator=g)[:P] for _ in range(B)])
        x = {"input_ids": ids, "masked_positions": mpos, "token_type_ids": torch.zeros_like(ids),
             "attention_mask": torch.ones(B, S)}
        batches.append((x, torch.randint(0, V, (B, P), generator=g)))
    batches = batches * 5

    def model_fn():
        initializers.set_seed(12)
        return BertModel(vocab=V, hidden=128, layers=2, heads=2, ffn=256, max_pos=S, dropout=0.0)

    def opt_fn():
        return optimizers.AdamW(1e-3, weight_decay=0.01, epsilon=1e-6)

    gl, gw = _train(model_fn, opt_fn, batches, cuda)
    cl, cw = _train(model_fn, opt_fn, batches, torch.device("cpu"))
    assert all(np.isfinite(gl)) and gl[-1] < gl[0], gl
    for a, b in zip(gl, cl):
        assert abs(a - b) <= 0.02 * abs(b) + 0.02, (gl, cl)
    worst = max((_rel(gw[k], cw[k]), k) for k in cw if cw[k].size > 1 and np.linalg.norm(cw[k]) > 0)
    assert worst[0] < 0.05, worst



def test_gpt2_tiny_fp8_trains_like_bf16(cuda):
    """The fp8 configuration of BASELINE.json:11 on a tiny GPT-2: every projection GEMM on the block-scaled fp8 MFMA
    (e4m3 x e4m3 forward, e5m2 x e4m3 backward, delayed per-tensor scaling) against the same model, initial weights
    and batches in bf16. 30 AdamW steps over 3 revisited batches: the loss curves must agree within 5% at every step
    and both must learn (a whole-model fp8 test)."""
    from distributed_tensorflow_amd.models.transformer import GPT2
    g = torch.Generator().manual_seed(4)
    V, S, B = 512, 128, 4
    batches = [(torch.randint(0, V, (B, S), generator=g), None) for _ in range(3)]
    batches = [(x, torch.roll(x, -1, 1)) for x, _ in batches] * 10

    def run(fp8):
        def model_fn():
            initializers.set_seed(21)
            return GPT2(vocab=V, ctx=S, hidden=256, layers=2, heads=4, dropout=0.0, fp8=fp8)

        def opt_fn():
            return optimizers.AdamW(1e-3, weight_decay=0.01)
        return _train(model_fn, opt_fn, batches, cuda)

    l8, _ = run(True)
    lb, _ = run(False)
    assert all(np.isfinite(l8)), l8
    for a, b in zip(l8, lb):
        assert abs(a - b) <= 0.05 * abs(b), (l8, lb)
    assert l8[-1] < 0.8 * l8[0] and lb[-1] < 0.8 * lb[0], (l8, lb)
