"""Reference-point / weight sampling (reference ``operators/sampling/*.py``)."""
from __future__ import annotations

from itertools import combinations
from math import comb

import torch

from ...ops import random as rnd


def _das_dennis(h: int, m: int) -> torch.Tensor:
    c = torch.tensor(list(combinations(range(1, h + m), m - 1)), dtype=torch.float32)
    c = c - torch.arange(m - 1, dtype=torch.float32)[None, :] - 1
    w = torch.cat([c, torch.full((c.shape[0], 1), float(h))], 1) - torch.cat([torch.zeros((c.shape[0], 1)), c], 1)
    return w / h


class UniformSampling:
    """Das–Dennis (two-layer when needed) simplex lattice, PlatEMO's NBI."""

    def __init__(self, n=None, m=None):
        self.n, self.m = n, m

    def __call__(self, key=None):
        n, m = self.n, self.m
        h1 = 1
        while comb(h1 + m, m - 1) <= n:
            h1 += 1
        w = _das_dennis(h1, m)
        if h1 < m:
            h2 = 0
            while comb(h1 + m - 1, m - 1) + comb(h2 + m, m - 1) <= n:
                h2 += 1
            if h2 > 0:
                w2 = _das_dennis(h2, m)
                w = torch.cat([w, w2 / 2.0 + 1.0 / (2.0 * m)], 0)
        w = torch.clamp(w, min=1e-6)
        return w, w.shape[0]


class LatinHypercubeSampling:
    def __init__(self, n=None, m=None):
        self.n, self.m = n, m

    def __call__(self, key):
        ks = rnd.split(key, self.m + 1)
        w = rnd.uniform(ks[0], (self.n, self.m))
        parm = torch.stack([rnd.permutation(ks[i + 1], self.n) for i in range(self.m)], 1).to(torch.float32) + 1
        return (parm - w) / self.n, self.n


class GridSampling:
    def __init__(self, n=None, m=None):
        self.n, self.m = n, m
        self.num_points = int(torch.ceil(torch.tensor(n ** (1 / m))).item())

    def __call__(self):
        gap = torch.linspace(0, 1, self.num_points)
        grids = torch.meshgrid(*[gap] * self.m, indexing="ij")
        w = torch.stack(grids, -1).reshape(-1, self.m).flip(1)
        return w, w.shape[0]
