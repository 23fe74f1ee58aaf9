"""Population reductions (``reduce.hip``)."""
from __future__ import annotations

import torch

from . import _ext


def weighted_rowsum(X: torch.Tensor, idx, w: torch.Tensor, sub, K: int) -> torch.Tensor:
    """``Σ_{k<K} w[k] (X[idx[k]] − sub)`` → (d,) (``idx=None`` ⇒ rows 0..K−1)."""
    if X.is_cuda:
        i = None if idx is None else idx.to(torch.int32).contiguous()
        return _ext.ops().weighted_rowsum(X, i, w.contiguous(), None if sub is None else sub.contiguous(), int(K))
    rows = X[idx[:K].long()] if idx is not None else X[:K]
    if sub is not None:
        rows = rows - sub
    return w[:K] @ rows
