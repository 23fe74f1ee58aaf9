"""State write-back helper of the hipGraph path (evoxmi/runtime/graph.py:copy_into): mixed-dtype
leaves are moved as 32-bit words in one multi-tensor copy, odd-sized dtypes one by one."""
import torch

from evoxmi.runtime.graph import copy_into


def test_copy_into_mixed_dtypes_matches_per_tensor_copy():
    g = torch.Generator().manual_seed(0)
    src = [torch.randn(5, generator=g), torch.tensor(7), torch.randn(3, dtype=torch.float64, generator=g),
           torch.tensor([True, False, True]), torch.randn(4, 4, generator=g), torch.tensor(2.5),
           torch.randint(0, 9, (6,), dtype=torch.int32, generator=g), torch.zeros(0)]
    dst = [torch.empty_like(s) for s in src]
    copy_into(dst, src)
    for d, s in zip(dst, src):
        assert d.dtype == s.dtype and torch.equal(d, s)


def test_copy_into_same_dtype_and_single_pair():
    src = [torch.arange(4.0), torch.arange(3.0)]
    dst = [torch.zeros(4), torch.zeros(3)]
    copy_into(dst, src)
    assert torch.equal(dst[0], src[0]) and torch.equal(dst[1], src[1])
    one = torch.zeros(2, dtype=torch.int64)
    copy_into([one], [torch.tensor([3, 4])])
    assert one.tolist() == [3, 4]
