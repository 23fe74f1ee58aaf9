"""Device launchers for benchmark-problem kernels (classic, CEC2022, DTLZ, LSMOP)."""
from __future__ import annotations

import torch

from . import _ext


def classic_eval(X: torch.Tensor, func_id: int, a: float = 0.0, b: float = 0.0, c: float = 0.0) -> torch.Tensor:
    X = X.contiguous()
    return _ext.ops().classic_eval(X, int(func_id), float(a), float(b), float(c))


def cec_basic(Z, fid, perm=None, start=0, L=None, sub=None, scale=1.0, Y=None, ystart=0, yperm=False, clamp=0.0):
    L = Z.shape[1] - start if L is None else L
    p = None if perm is None else perm.to(torch.int32).contiguous()
    s = None if sub is None else sub.contiguous()
    return _ext.ops().cec_basic(Z, int(fid), p, int(start), int(L), s, float(scale), Y, int(ystart), int(yperm), float(clamp))


def dtlz(X, m, variant):
    """Fused DTLZ1–4 objectives (``csrc/kernels/mo_problems.hip``), X: (n, d) f32 on GPU."""
    return _ext.ops().dtlz(X.contiguous(), int(m), int(variant))
