"""Direct accumulation of parameter gradients into the arena (ops._util.direct_grads, used by
Model.train_step) must produce exactly what the regular autograd AccumulateGrad path produces, including
accumulation over several backward passes, and must keep the post-accumulate hooks (gradient bucketing)
firing once per parameter per backward."""
import pytest
import torch

from distributed_tensorflow_amd import ops
from distributed_tensorflow_amd.ops._util import direct_grads
from distributed_tensorflow_amd.variables import ParamArena, Variable

BF = torch.bfloat16


def _run(dev, direct):
    torch.manual_seed(11)
    V, S, B, D, F = 96, 32, 4, 64, 128
    word = Variable(torch.randn(V, D) * 0.1, name="word")
    pos = Variable(torch.randn(S, D) * 0.1, name="pos")
    typ = Variable(torch.randn(2, D) * 0.1, name="typ")
    g = Variable(torch.rand(D) + 0.5, name="ln/gamma")
    b = Variable(torch.zeros(D), name="ln/beta")
    w1 = Variable(torch.randn(F, D) * 0.05, name="w1")
    b1 = Variable(torch.zeros(F), name="b1")
    w2 = Variable(torch.randn(D, F) * 0.05, name="w2")
    params = [word, pos, typ, g, b, w1, b1, w2]
    for p in params:
        p.data = p.data.to(dev)
    arena = ParamArena(params, device=dev)
    fired = []
    for p in params:
        p.register_post_accumulate_grad_hook(lambda t: fired.append(t.name))
    ids = torch.randint(0, V, (B, S), device=dev)
    tids = torch.randint(0, 2, (B, S), device=dev)
    for _ in range(2):
        h = ops.embedding(ids, word, pos, tids, typ)
        h = ops.layer_norm(h, g, b, 1e-5)
        y = ops.dense(ops.dense(h, w1, b1, act="gelu"), w2)
        loss = y.float().square().mean()
        if direct:
            with direct_grads():
                loss.backward()
        else:
            loss.backward()
    assert sorted(fired) == sorted([p.name for p in params] * 2)
    return arena.grad.clone()


@pytest.mark.gpu
def test_transformer_ops_direct_grads(cuda):
    a = _run(cuda, False)
    d = _run(cuda, True)
    err = (a - d).abs().max().item()
    assert err <= 1e-5 * (a.abs().max().item() + 1e-6), err


def test_direct_grads_cpu_is_noop():
    """CPU ops use the torch reference path; direct mode changes nothing there."""
    a = _run(torch.device("cpu"), False)
    d = _run(torch.device("cpu"), True)
    assert torch.equal(a, d)
