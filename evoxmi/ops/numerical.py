"""Device launchers for benchmark-problem kernels (classic, CEC2022, DTLZ, LSMOP)."""
from __future__ import annotations

import torch

from . import _ext


def classic_eval(X: torch.Tensor, func_id: int, a: float = 0.0, b: float = 0.0, c: float = 0.0) -> torch.Tensor:
    X = X.contiguous()
    return _ext.ops().classic_eval(X, int(func_id), float(a), float(b), float(c))
