"""Inverted generational distance IGD and IGD+ (reference ``metrics/igd.py:7-41``)."""
from __future__ import annotations

import torch

from ..ops import geom
from .gd import _plus_dist


def igd(objs, pf, p=1):
    objs, pf = objs.to(torch.float32), pf.to(torch.float32).to(objs.device)
    m = geom.min_dist(pf, objs)  # fused nearest-row kernel on the GPU (K17)
    return ((m**p).sum() / pf.shape[0]) ** (1 / p)


def igd_plus(objs, pf, p=1):
    objs, pf = objs.to(torch.float32), pf.to(torch.float32).to(objs.device)
    m = _plus_dist(objs, pf).T.min(1).values  # ‖max(obj − z, 0)‖ for each reference point z
    return ((m**p).sum() / pf.shape[0]) ** (1 / p)


class IGD:
    def __init__(self, pf, p=1):
        self.pf, self.p = pf, p

    def __call__(self, objs):
        return igd(objs, self.pf, self.p)


class IGDPlus:
    def __init__(self, pf, p=1):
        self.pf, self.p = pf, p

    def __call__(self, objs):
        return igd_plus(objs, self.pf, self.p)
