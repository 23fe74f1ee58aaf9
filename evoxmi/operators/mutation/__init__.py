"""Mutation operators (reference ``operators/mutation/*.py``)."""
from __future__ import annotations

import torch

from ...ops import random as rnd


def polynomial(key, x, boundary, pro_m=1.0, dis_m=20.0, cols=None):
    """PlatEMO polynomial mutation; per-gene probability ``pro_m / d``; an odd last row passes through.

    ``cols = (col0, d_total)``: ``x`` and ``boundary`` are the column block [col0, col0 + d) of
    a d_total-dim problem; the site probability is ``pro_m / d_total`` and the draws are
    those of the global columns."""
    if x.is_cuda and x.dtype == torch.float32 and x.shape[0] > 1:
        from ...ops import evo as evo_ops

        return evo_ops.polynomial(key, x, boundary[0], boundary[1], float(pro_m), float(dis_m), cols)
    k1, k2 = rnd.split(key)
    pop = x if x.shape[0] == 1 else x[: (x.shape[0] // 2) * 2]
    n, d = pop.shape
    dev = x.device
    c0, dt = cols if cols is not None else (0, d)
    site = rnd.uniform(k1, (n, dt)).to(dev)[:, c0 : c0 + d] < pro_m / dt
    mu = rnd.uniform(k2, (n, dt)).to(dev)[:, c0 : c0 + d]
    lower = boundary[0].to(dev).expand(n, d)
    upper = boundary[1].to(dev).expand(n, d)
    pop = torch.maximum(torch.minimum(pop, upper), lower)
    temp = site & (mu <= 0.5)
    norm = torch.where(temp, (pop - lower) / (upper - lower), torch.zeros_like(pop))
    pop = torch.where(temp, pop + (upper - lower) * ((2.0 * mu + (1.0 - 2.0 * mu) * (1.0 - norm) ** (dis_m + 1.0)) ** (1.0 / (dis_m + 1)) - 1.0), pop)
    temp = site & (mu > 0.5)
    norm = torch.where(temp, (upper - pop) / (upper - lower), torch.zeros_like(pop))
    pop = torch.where(temp, pop + (upper - lower) * (1.0 - (2.0 * (1.0 - mu) + 2.0 * (mu - 0.5) * (1.0 - norm) ** (dis_m + 1.0)) ** (1.0 / (dis_m + 1.0))), pop)
    if x.shape[0] % 2 != 0 and x.shape[0] != 1:
        pop = torch.cat([pop, x[-1:]], 0)
    return pop


class Polynomial:
    column_blocks = True  # accepts cols= and a column-block boundary

    def __init__(self, boundary, pro_m=1, dis_m=20):
        self.boundary, self.pro_m, self.dis_m = boundary, pro_m, dis_m

    def __call__(self, key, x, cols=None, boundary=None):
        return polynomial(key, x, self.boundary if boundary is None else boundary, self.pro_m, self.dis_m, cols)


def gaussian(key, x, stdvar):
    return x + rnd.normal(key, x.shape).to(x.device) * stdvar


class Gaussian:
    def __init__(self, stdvar=1.0):
        self.stdvar = stdvar

    def __call__(self, key, x):
        return gaussian(key, x, self.stdvar)


def bitflip(key, x, prob, bool_input="auto"):
    """Bit-flip on a bool tensor, or on packed uint8 bits (8 flips per byte)."""
    if bool_input == "auto":
        if x.dtype == torch.bool:
            bool_input = True
        elif x.dtype == torch.uint8:
            bool_input = False
        else:
            raise TypeError("The input x should be type bool or uint8")
    if bool_input:
        return x ^ (rnd.uniform(key, x.shape).to(x.device) < prob)
    flips = (rnd.uniform(key, (*x.shape, 8)).to(x.device) < prob).to(torch.uint8)
    weights = torch.tensor([128, 64, 32, 16, 8, 4, 2, 1], dtype=torch.uint8, device=x.device)
    packed = (flips * weights).sum(-1).to(torch.uint8)
    return x ^ packed


class Bitflip:
    def __init__(self, prob, bool_input="auto"):
        self.prob, self.bool_input = prob, bool_input

    def __call__(self, key, x):
        return bitflip(key, x, self.prob, self.bool_input)
