"""Sorting primitives (K19).  Device path: one-workgroup LDS radix argsort (rocPRIM block
radix sort, ``sort.hip``) for n ≤ 4096 — one launch, no workspace; larger inputs use the
ROCm library radix sort, which spreads over the CUs.  Measured on MI355X
(profiles/r2_sort_microbench.log, µs per call): n = 1000: radix 10.7 / bitonic 11.2 /
library 21.0; n = 4096: 21.3 / 31.5 / 31.7; n = 10 000: 43.9 / 119.8 / 32.5 — one
workgroup stops paying off above ≈4k keys.  Ties are broken by index (== stable sort)."""
from __future__ import annotations

import torch

from . import _ext

MAX_LDS_SORT = 4096


def argsort(keys: torch.Tensor, descending: bool = False):
    """Return ``(sorted_keys, indices[int64])`` of a 1-D float tensor."""
    if keys.is_cuda and keys.dtype == torch.float32 and keys.numel() <= MAX_LDS_SORT:
        k, i = _ext.ops().radix_argsort_f32(keys.contiguous(), int(descending))
        return k, i.long()
    v, i = torch.sort(keys, descending=descending, stable=True)
    return v, i


def argsort_i32(keys: torch.Tensor):
    """Ascending argsort returning int32 indices (feeds gather prologues directly)."""
    if keys.is_cuda and keys.dtype == torch.float32 and keys.numel() <= MAX_LDS_SORT:
        return _ext.ops().radix_argsort_f32(keys.contiguous(), 0)
    v, i = torch.sort(keys, stable=True)
    return v, i.to(torch.int32)


def topk(x: torch.Tensor, k: int, dim: int = -1, largest: bool = True):
    """hipGraph-capture-safe top-k → (values, indices), sorted.

    ``torch.topk`` on ROCm returns corrupted indices when replayed from a captured
    hipGraph (observed on MI355X / torch 2.10+rocm7.0: the index buffer aliases a
    float workspace), so every capturable code path uses this instead: k rounds of
    arg-max with masking for small k, a stable argsort otherwise.
    """
    if dim != -1 and dim != x.ndim - 1:
        v, i = topk(x.transpose(dim, -1), k, -1, largest)
        return v.transpose(dim, -1), i.transpose(dim, -1)
    n = x.shape[-1]
    k = min(k, n)
    if k <= 8:
        work = x.clone() if largest else -x
        fill = float("-inf") if work.is_floating_point() else torch.iinfo(work.dtype).min
        idx = []
        for _ in range(k):
            j = torch.argmax(work, dim=-1, keepdim=True)
            idx.append(j)
            work = work.scatter(-1, j, fill)  # out of place: also runs under vmap
        ind = torch.cat(idx, -1)
    else:
        ind = torch.argsort(x, dim=-1, descending=largest, stable=True)[..., :k]
    return torch.gather(x, -1, ind), ind
