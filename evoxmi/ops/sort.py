"""Sorting primitives (K19).  Device path: LDS bitonic argsort in one workgroup for
n ≤ 16384 (the population sizes of every north-star config); larger inputs use
the ROCm library sort.  Ties are broken by index (== stable sort)."""
from __future__ import annotations

import torch

from . import _ext

MAX_LDS_SORT = 16384


def argsort(keys: torch.Tensor, descending: bool = False):
    """Return ``(sorted_keys, indices[int64])`` of a 1-D float tensor."""
    if keys.is_cuda and keys.dtype == torch.float32 and keys.numel() <= MAX_LDS_SORT:
        k, i = _ext.ops().argsort_f32(keys.contiguous(), int(descending))
        return k, i.long()
    v, i = torch.sort(keys, descending=descending, stable=True)
    return v, i


def argsort_i32(keys: torch.Tensor):
    """Ascending argsort returning int32 indices (feeds gather prologues directly)."""
    if keys.is_cuda and keys.dtype == torch.float32 and keys.numel() <= MAX_LDS_SORT:
        return _ext.ops().argsort_f32(keys.contiguous(), 0)
    v, i = torch.sort(keys, stable=True)
    return v, i.to(torch.int32)
