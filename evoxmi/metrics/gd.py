"""Generational distance GD and GD+ (reference ``metrics/gd.py:7-41``).

``GD_p = (Σ_i min_j d(x_i, z_j)^p / |X|)^{1/p}``; the nearest distances come from the
fused nearest-row kernel (``ops.geom.min_dist``, K17); GD+ uses the modified distance
‖max(x − z, 0)‖ (Ishibuchi et al. 2015).
"""
from __future__ import annotations

import torch

from ..ops import geom


def _plus_dist(a, b):
    """‖max(a_i − b_j, 0)‖ for all pairs, (|a|, |b|)."""
    return torch.sqrt((torch.clamp(a[:, None, :] - b[None, :, :], min=0) ** 2).sum(-1))


def gd(objs, pf, p=1):
    objs, pf = objs.to(torch.float32), pf.to(torch.float32).to(objs.device)
    m = geom.min_dist(objs, pf)
    return ((m**p).sum() / objs.shape[0]) ** (1 / p)


def gd_plus(objs, pf, p=1):
    objs, pf = objs.to(torch.float32), pf.to(torch.float32).to(objs.device)
    # reference gd_plus_dist(pf, obj) = ‖max(pf − obj, 0)‖ evaluated as pairwise_func(objs, pf, ·)
    m = _plus_dist(objs, pf).min(1).values
    return ((m**p).sum() / objs.shape[0]) ** (1 / p)


class GD:
    def __init__(self, pf, p=1):
        self.pf, self.p = pf, p

    def __call__(self, objs):
        return gd(objs, self.pf, self.p)


class GDPlus:
    def __init__(self, pf, p=1):
        self.pf, self.p = pf, p

    def __call__(self, objs):
        return gd_plus(objs, self.pf, self.p)
