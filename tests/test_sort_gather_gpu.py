"""The radix sort and indexed row gather of csrc/kernels/sort.hip (the embedding-gradient sort and
the masked-LM gather ran rocPRIM / aten kernels): exact against torch's stable sort and index_select, the gather
gradient against an f32 index_add reference, and both bitwise reproducible."""
import pytest
import torch

from distributed_tensorflow_amd import ops
from distributed_tensorflow_amd.ops import _util

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n,hi,bits", [(1, 5, 3), (1000, 50, 6), (1024, 30522, 15), (65536 + 17, 30522, 15),
                                       (200000, 50257, 16), (4099, 2, 1), (7000, 1 << 20, 21)])
def test_sort_keys_matches_stable_sort(cuda, n, hi, bits):
    g = torch.Generator().manual_seed(n)
    k = torch.randint(0, hi, (n,), generator=g).to(cuda)
    with _util.call_log() as log:
        sk, perm = ops.sort_keys(k, bits)
    assert log["dtf_sort_keys"] == 1
    rk, rp = torch.sort(k.cpu(), stable=True)
    assert torch.equal(sk.cpu(), rk) and torch.equal(perm.cpu(), rp)
    sk2, perm2 = ops.sort_keys(k, bits)
    assert torch.equal(perm2, perm)


def test_gather_rows_forward_backward(cuda):
    g = torch.Generator().manual_seed(0)
    R, D, n = 4096, 768, 3000
    src = torch.randn(R, D, generator=g).to(cuda, torch.bfloat16).requires_grad_(True)
    idx = torch.randint(0, R // 2, (n,), generator=g).to(cuda)  # duplicates, and rows nobody gathers
    dy = torch.randn(n, D, generator=g).to(cuda, torch.bfloat16)
    with _util.call_log() as log:
        out = ops.gather_rows(src, idx)
        out.backward(dy)
    assert log["dtf_gather_rows"] == 1 and log["dtf_gather_rows_bwd"] == 1 and log["dtf_sort_keys"] == 1
    assert torch.equal(out, src.detach().index_select(0, idx))
    ref = torch.zeros(R, D, dtype=torch.float32, device=cuda).index_add_(0, idx, dy.float())
    torch.testing.assert_close(src.grad.float(), ref, rtol=1e-2, atol=2e-2)
    assert not src.grad[R // 2:].any()
    g1 = src.grad.clone()
    src.grad = None
    ops.gather_rows(src, idx).backward(dy)
    assert torch.equal(src.grad, g1)  # deterministic
