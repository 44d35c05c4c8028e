"""The flagship train steps run on OUR kernels, not on a vendor library.

* A TorchDispatchMode guard fails on any aten GEMM / convolution (mm, addmm, bmm, baddbmm, _scaled_mm, convolution,
  ...) with a CUDA operand — the round-4 hipBLASLt routes (torch.mm / F.linear / torch._scaled_mm) are exactly what it
  catches. It runs over a whole ResNet-50 training step and a GPT-2 (bf16 and fp8) training step.
* It also fails on the aten sort / indexed-row ops (sort, index_select, index_add, scatter_add, gather, ...) with a
  CUDA operand: the embedding gradient's sort and the masked-LM gather run csrc/kernels/sort.hip,
  checked over a BERT-base-shaped MLM step too.
* The GEMM dispatch's host-side launch counters (csrc/kernels/common.h LaunchCounter) show which kernel a call reached,
  so these steps are also pinned to the hand-written 4-wave GEMM (gemm_w4.hip) where the dense layers should land.
Dispatch modes are thread-local state that autograd propagates to its backward threads, so the backward is covered.
"""
import pytest
import torch
from torch.utils._python_dispatch import TorchDispatchMode

from distributed_tensorflow_amd.keras import initializers, losses, optimizers
from distributed_tensorflow_amd.ops import _util

pytestmark = pytest.mark.gpu

_BANNED = {"mm", "addmm", "bmm", "baddbmm", "_scaled_mm", "convolution", "_convolution", "cudnn_convolution",
           "miopen_convolution", "convolution_backward", "matmul", "linear", "addmv", "mv", "_int_mm", "addbmm",
           "sort", "argsort", "index_select", "index_add", "index_add_", "scatter_add", "scatter_add_", "gather",
           "index", "index_put", "index_put_", "embedding", "embedding_dense_backward", "unique", "_unique2"}


class NoLibraryGemm(TorchDispatchMode):
    """Records every banned aten op that touches a CUDA tensor."""

    def __init__(self):
        super().__init__()
        self.hits = []

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        kwargs = kwargs or {}
        name = func.overloadpacket.__name__
        if name in _BANNED:
            flat = list(args) + list(kwargs.values())
            if any(isinstance(t, torch.Tensor) and t.is_cuda for t in flat):
                self.hits.append(str(func))
        return func(*args, **kwargs)


def _step(model_fn, opt, x, y, dev):
    from distributed_tensorflow_amd import context
    with context.device(dev):
        m = model_fn()
        m.compile(optimizer=opt, loss=losses.SparseCategoricalCrossentropy(from_logits=True))
        m.train_step((x, y))  # builds the lazy weights, bf16 shadows, fp8 scales
        torch.cuda.synchronize()
        before = _util.launch_counts()
        with NoLibraryGemm() as guard:
            logs = m.train_step((x, y))
            torch.cuda.synchronize()
        return float(logs["loss"]), guard.hits, _util.launch_delta(before)


def test_guard_catches_a_library_gemm(cuda):
    """The guard itself: torch.mm / F.linear on CUDA tensors are reported, CPU ones are not."""
    a = torch.randn(64, 64, device=cuda, dtype=torch.bfloat16)
    with NoLibraryGemm() as g:
        torch.mm(a, a)
        torch.nn.functional.linear(a, a)
        torch.mm(a.cpu().float(), a.cpu().float())
    assert len(g.hits) == 2, g.hits


def test_resnet50_step_runs_no_library_gemm(cuda):
    from distributed_tensorflow_amd.models import ResNet
    torch.manual_seed(0)
    x = torch.randn(8, 3, 224, 224, device=cuda)
    y = torch.randint(0, 1000, (8,), device=cuda)
    loss, hits, delta = _step(lambda: ResNet(50, num_classes=1000), optimizers.SGD(0.01, momentum=0.9), x, y, cuda)
    assert loss == loss
    assert not hits, f"library GEMM / conv on the ResNet-50 step: {hits[:5]}"


@pytest.mark.parametrize("fp8", [False, True])
def test_gpt2_step_runs_our_gemms(cuda, fp8):
    from distributed_tensorflow_amd.models.transformer import GPT2
    g = torch.Generator().manual_seed(1)
    V, S, B = 1024, 256, 8
    x = torch.randint(0, V, (B, S), generator=g).to(cuda)
    y = torch.roll(x, -1, 1)

    def model_fn():
        initializers.set_seed(3)
        return GPT2(vocab=V, ctx=S, hidden=512, layers=2, heads=8, dropout=0.0, fp8=fp8)

    loss, hits, delta = _step(model_fn, optimizers.AdamW(1e-4), x, y, cuda)
    assert loss == loss
    assert not hits, f"library GEMM on the GPT-2 step: {hits[:5]}"
    if not fp8:  # the bf16 projections (2048 tokens x 512..2048) land on the 4-wave kernel
        assert delta["w4_256"] + delta["w4_128"] >= 8, delta


def test_bert_mlm_step_runs_our_kernels(cuda):
    """A BERT-base-shaped MLM step (12 heads, 768 hidden, masked positions gathered): no library GEMM, no aten sort or
    indexed-row op — the word-embedding gradient sorts with dtf_sort_keys, the MLM gather is dtf_gather_rows."""
    from distributed_tensorflow_amd.models.transformer import BertModel
    g = torch.Generator().manual_seed(2)
    B, S, P, V = 4, 128, 20, 30522
    ids = torch.randint(0, V, (B, S), generator=g).to(cuda)
    mpos = torch.stack([torch.randperm(S, generator=g)[:P] for _ in range(B)]).to(cuda)
    lab = torch.randint(0, V, (B, P), generator=g).to(cuda)
    x = {"input_ids": ids, "masked_positions": mpos, "token_type_ids": torch.zeros_like(ids),
         "attention_mask": torch.ones(B, S, device=cuda)}

    def model_fn():
        initializers.set_seed(4)
        return BertModel(layers=2)

    with _util.call_log() as log:
        loss, hits, delta = _step(model_fn, optimizers.AdamW(1e-4), x, lab, cuda)
    assert loss == loss
    assert not hits, f"library / aten indexed op on the BERT step: {hits[:5]}"
    assert log["dtf_sort_keys"] >= 2 and log["dtf_gather_rows"] >= 2 and log["dtf_gather_rows_bwd"] >= 2, log
