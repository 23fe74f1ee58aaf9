"""Sorting primitives (K19).  Device path for n ≤ 16384 (every population size of the
north-star configs): the rank-by-counting argsort of ``sort.hip`` — all keys in LDS, each
256-thread workgroup ranks 64 elements against all n keys, one launch, no workspace, and
n/64 workgroups spread over the CUs (the single-workgroup radix/bitonic kernels cannot:
round 2 measured them at 43.9 / 119.8 µs for n = 10 000 against the library's 32.5,
profiles/r2_sort_microbench.log).  Larger inputs use the ROCm library radix sort.  Ties are
broken by index (== stable sort); NaN sorts as the largest key and −0.0 ties with +0.0, as
in ``torch.sort``.  Numbers: ``tools/bench_sort.py`` → profiles/r3_sort_microbench.log."""
from __future__ import annotations

import torch

from . import _ext

MAX_RANK_SORT = 16384


def _device(keys):
    return keys.is_cuda and keys.dtype == torch.float32 and keys.dim() <= 2 and keys.shape[-1] <= MAX_RANK_SORT


def argsort(keys: torch.Tensor, descending: bool = False):
    """Return ``(sorted_keys, indices[int64])`` along the last dim of a 1-D or (B, n) float tensor."""
    if _device(keys):
        k, i = _ext.ops().rank_argsort_f32(keys.contiguous(), int(descending))
        return k, i.long()
    v, i = torch.sort(keys, descending=descending, stable=True)
    return v, i


def argsort_i32(keys: torch.Tensor):
    """Ascending argsort returning int32 indices (feeds gather prologues directly)."""
    if _device(keys):
        return _ext.ops().rank_argsort_f32(keys.contiguous(), 0)
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
