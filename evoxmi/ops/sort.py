"""Sorting primitives (K19).  Device path for n ≤ 16384 (every population size of the
north-star configs): the rank-by-counting argsort of ``sort.hip`` — all keys in LDS, each
256-thread workgroup ranks 64 elements against all n keys, one launch, no workspace, and
n/64 workgroups spread over the CUs (the single-workgroup radix/bitonic kernels cannot:
round 2 measured them at 43.9 / 119.8 µs for n = 10 000 against the library's 32.5,
profiles/r2_sort_microbench.log).  From 8192 to 32768 keys the two-pass merge sort takes over:
rank inside 4096-key chunks, then place every element by lockstep binary searches of the other
sorted chunks staged in LDS (17.4 µs at 16 384, 33 µs at 30 000 against torch.sort's 32.8 / 42.6;
reference primitives: src/evox/algorithms/so/es_variants/sort_utils.py:5-12,
src/evox/operators/selection/topk_fit.py:7-12).  Larger inputs use the ROCm library radix sort.  Ties are
broken by index (== stable sort); NaN sorts as the largest key and −0.0 ties with +0.0, as
in ``torch.sort``.  Numbers: ``tools/bench_sort.py`` → profiles/r3_sort_microbench.log."""
from __future__ import annotations

import torch

from . import _ext

MAX_RANK_SORT = 8192     # one-launch rank-by-counting up to here (profiles/r3_sort_microbench.log)
MAX_DEVICE_SORT = 32768  # two-pass merge up to here; the library radix sort beyond


def _batched(x) -> bool:
    """Inside ``torch.vmap`` (BatchedRuns): the custom ops carry no batching rule there."""
    try:
        return bool(torch._C._functorch.is_batchedtensor(x))
    except AttributeError:  # pragma: no cover - older torch
        return False


def _device(keys):
    return (keys.is_cuda and keys.dtype == torch.float32 and 1 <= keys.dim() <= 2 and keys.shape[-1] <= MAX_DEVICE_SORT
            and not _batched(keys))


def _sort(keys, descending):
    ops = _ext.ops()
    fn = ops.rank_argsort_f32 if keys.shape[-1] <= MAX_RANK_SORT else ops.merge_argsort_f32
    return fn(keys.contiguous(), int(descending))


def argsort(keys: torch.Tensor, descending: bool = False):
    """Return ``(sorted_keys, indices[int64])`` along the last dim of a 1-D or (B, n) float tensor."""
    if _device(keys):
        k, i = _sort(keys, descending)
        return k, i.long()
    v, i = torch.sort(keys, descending=descending, stable=True)
    return v, i


def argsort_i32(keys: torch.Tensor):
    """Ascending argsort returning int32 indices (feeds gather prologues directly)."""
    if _device(keys):
        return _sort(keys, False)
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
    elif _device(x):
        ind = argsort(x, descending=largest)[1][..., :k]
    else:
        ind = torch.argsort(x, dim=-1, descending=largest, stable=True)[..., :k]
    return torch.gather(x, -1, ind), ind
