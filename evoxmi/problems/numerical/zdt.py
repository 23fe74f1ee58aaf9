"""ZDT1–4, 6 (reference ``problems/numerical/zdt.py:14-100``): 2 objectives
(f1, g·h(f1, g)); analytic ``pf()``."""
from __future__ import annotations

import math

import torch

from ...core import Problem


class ZDTTestSuit(Problem):
    def __init__(self, n, ref_num=100):
        super().__init__()
        self.n, self.ref_num = n, ref_num

    def _f1(self, X):
        return X[:, 0]

    def _g(self, X):
        return self._g_from(self._g_partial(X[:, 1:]))

    def _g_partial(self, Y):
        return Y.sum(1)

    def _g_from(self, S):
        return 1 + 9 * S / (self.n - 1)

    # -- decision-axis sharding (P2, evoxmi/parallel/dim_sharded.py): x_1 from its owner and
    # the additive part of g
    dim_halo = 0

    def partial_terms(self, Xb, col0, d, own):
        Xo = Xb[:, :own]
        T = torch.zeros((Xb.shape[0], 2), dtype=Xb.dtype, device=Xb.device)
        if col0 == 0 and own > 0:
            T[:, 0] = Xo[:, 0]
        s = max(1 - col0, 0)
        if s < own:
            T[:, 1] = self._g_partial(Xo[:, s:])
        return T

    def combine_terms(self, T, d):
        f1 = self._f1(T[:, :1])
        g = self._g_from(T[:, 1])
        return torch.stack([f1, g * self._h(f1, g)], 1)

    def _h(self, f1, g):
        return 1 - torch.sqrt(f1 / g)

    def evaluate(self, state, X):
        f1 = self._f1(X)
        g = self._g(X)
        return torch.stack([f1, g * self._h(f1, g)], 1), state

    def pf(self):
        x = torch.linspace(0, 1, self.ref_num)
        return torch.stack([x, 1 - torch.sqrt(x)], 1)


class ZDT1(ZDTTestSuit):
    pass


class ZDT2(ZDTTestSuit):
    def _h(self, f1, g):
        return 1 - (f1 / g) ** 2

    def pf(self):
        x = torch.linspace(0, 1, self.ref_num)
        return torch.stack([x, 1 - x**2], 1)


class ZDT3(ZDTTestSuit):
    def _h(self, f1, g):
        return 1 - torch.sqrt(f1 / g) - (f1 / g) * torch.sin(10 * math.pi * f1)

    def pf(self):
        r = torch.tensor([[0, 0.0830], [0.1822, 0.2577], [0.4093, 0.4538], [0.6183, 0.6525], [0.8233, 0.8518]])
        k = int(self.ref_num / len(r))
        f1 = torch.stack([torch.linspace(float(a), float(b), k) for a, b in r], 1)  # (k, 5)
        f2 = 1 - torch.sqrt(f1) - f1 * torch.sin(10 * math.pi * f1)
        return torch.stack([f1.T.reshape(-1), f2.T.reshape(-1)], 1)


class ZDT4(ZDTTestSuit):
    def _g_partial(self, Y):
        return (Y**2 - 10 * torch.cos(4 * math.pi * Y)).sum(1)

    def _g_from(self, S):
        return 1 + 10 * (self.n - 1) + S


class ZDT6(ZDTTestSuit):
    def _f1(self, X):
        return 1 - torch.exp(-4 * X[:, 0]) * torch.sin(6 * math.pi * X[:, 0]) ** 6

    def _g_from(self, S):
        return 1 + 9 * (S / 9) ** 0.25

    def _h(self, f1, g):
        return 1 - (f1 / g) ** 2

    def pf(self):
        f1 = torch.linspace(0.280775, 1, self.ref_num)
        return torch.stack([f1, 1 - f1**2], 1)
