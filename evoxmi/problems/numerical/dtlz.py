"""DTLZ1–7 (reference ``problems/numerical/dtlz.py:8-352``).

All objectives share the spherical/linear structure
``f = (1 + g) · fliplr(cumprod([1, h(x_{<m})])) · [1, t(x_{m-2::-1})]``; ``g`` is a
row reduction over the last d − m + 1 variables.  ``pf()`` samples the true
front with Das–Dennis points (``ref_num · m`` of them) as in the reference.
On a GPU the row reduction ``g`` and the m objectives of DTLZ1–4 are one fused
wave-per-row HIP kernel (``csrc/kernels/mo_problems.hip``).
"""
from __future__ import annotations

import math

import torch

from ...core import Problem, State
from ...operators.sampling import GridSampling, UniformSampling


def _cumprod_front(h: torch.Tensor, t: torch.Tensor):
    """fliplr(cumprod([1, h])) * [1, t_rev] — h: (n, m−1) factors, t: (n, m−1) last factors."""
    n = h.shape[0]
    ones = torch.ones((n, 1), dtype=h.dtype, device=h.device)
    a = torch.flip(torch.cumprod(torch.cat([ones, h], 1), 1), [1])
    b = torch.cat([ones, torch.flip(t, [1])], 1)
    return a * b


class DTLZTestSuit(Problem):
    def __init__(self, d, m, ref_num=1000):
        super().__init__()
        if d is None:
            raise ValueError("d must be specified, but got None")
        if m is None:
            raise ValueError("m must be specified, but got None")
        self.d, self.m, self.ref_num = d, m, ref_num
        self.sample = UniformSampling(self.ref_num * self.m, self.m)

    def setup(self, key):
        return State(key=key)

    def pf(self):
        return self.sample()[0] / 2

    # -- decision-axis sharding (P2, see evoxmi/parallel/dim_sharded.py): the m − 1 position
    # variables travel as terms (from the rank owning each column), the distance function g
    # is an additive row reduction over the last d − m + 1 variables
    dim_halo = 0

    def partial_terms(self, Xb, col0, d, own):
        m = self.m
        Xo = Xb[:, :own]
        T = torch.zeros((Xb.shape[0], m), dtype=Xb.dtype, device=Xb.device)
        hi = min(col0 + own, m - 1)
        if hi > col0:
            T[:, col0:hi] = Xo[:, : hi - col0]
        s = max(m - 1 - col0, 0)
        if s < own:
            T[:, m - 1] = self._g_partial(Xo[:, s:])
        return T

    def combine_terms(self, T, d):
        m = self.m
        return self._objectives(T[:, : m - 1], self._g_from(T[:, m - 1 :], d))

    def _g_partial(self, Y):
        return ((Y - 0.5) ** 2).sum(1)

    def _g_from(self, S, d):
        return S

    def evaluate(self, state, X):
        m = self.m
        return self._objectives(X[:, : m - 1], self._g_from(self._g_partial(X[:, m - 1 :])[:, None], X.shape[1])), state


def _spherical(X, m, g):
    h = torch.clamp(torch.cos(X[:, : m - 1] * math.pi / 2), min=0)
    t = torch.sin(X[:, : m - 1] * math.pi / 2)
    return (1 + g) * _cumprod_front(h, t)


def _rastrigin_g(X, m):
    d = X.shape[1]
    Y = X[:, m - 1 :] - 0.5
    return 100 * (d - m + 1 + (Y * Y - torch.cos(20 * math.pi * Y)).sum(1, keepdim=True))


def _fused(X, m, variant):
    if X.is_cuda and X.dtype == torch.float32 and m <= 64:
        from ...ops import numerical as nops

        return nops.dtlz(X, m, variant)
    return None


class DTLZ1(DTLZTestSuit):
    def __init__(self, d=None, m=None, ref_num=100):
        m = 3 if m is None else m
        d = m + 4 if d is None else d
        super().__init__(d, m, ref_num)

    def evaluate(self, state, X):
        r = _fused(X, self.m, 1)
        if r is not None:
            return r, state
        m = self.m
        return self._objectives(X[:, : m - 1], _rastrigin_g(X, m)), state

    _g_partial = staticmethod(lambda Y: ((Y - 0.5) ** 2 - torch.cos(20 * math.pi * (Y - 0.5))).sum(1))

    def _g_from(self, S, d):
        return 100 * (d - self.m + 1 + S)

    def _objectives(self, Xp, g):
        return 0.5 * (1 + g) * _cumprod_front(Xp, 1 - Xp)


class DTLZ2(DTLZTestSuit):
    def __init__(self, d=None, m=None, ref_num=1000):
        m = 3 if m is None else m
        d = m + 9 if d is None else d
        super().__init__(d, m, ref_num)

    def evaluate(self, state, X):
        r = _fused(X, self.m, 2)
        if r is not None:
            return r, state
        m = self.m
        g = ((X[:, m - 1 :] - 0.5) ** 2).sum(1, keepdim=True)
        return _spherical(X, m, g), state

    def _objectives(self, Xp, g):
        return _spherical(Xp, self.m, g)

    def pf(self):
        f = self.sample()[0]
        return f / torch.sqrt((f * f).sum(1, keepdim=True))


class DTLZ3(DTLZ2):
    def evaluate(self, state, X):
        r = _fused(X, self.m, 3)
        if r is not None:
            return r, state
        return _spherical(X, self.m, _rastrigin_g(X, self.m)), state

    _g_partial = staticmethod(DTLZ1._g_partial)
    _g_from = DTLZ1._g_from


class DTLZ4(DTLZ2):
    def evaluate(self, state, X):
        r = _fused(X, self.m, 4)
        if r is not None:
            return r, state
        m = self.m
        X = torch.cat([X[:, : m - 1] ** 100, X[:, m - 1 :]], 1)
        g = ((X[:, m - 1 :] - 0.5) ** 2).sum(1, keepdim=True)
        return _spherical(X, m, g), state

    def _objectives(self, Xp, g):
        return _spherical(Xp**100, self.m, g)


def _degenerate_pf(ref_num, m):
    n = ref_num * m
    a = torch.cat([torch.arange(0, 1, 1.0 / (n - 1)), torch.tensor([1.0])])
    b = torch.cat([torch.arange(1, 0, -1.0 / (n - 1)), torch.tensor([0.0])])
    k = min(a.shape[0], b.shape[0])
    f = torch.stack([a[:k], b[:k]], 1)
    f = f / torch.sqrt((f * f).sum(1, keepdim=True))
    for _ in range(m - 2):
        f = torch.cat([f[:, :1], f], 1)
    exps = torch.cat([torch.tensor([float(m - 2)]), torch.arange(m - 2, -1, -1, dtype=torch.float32)])
    return f / (math.sqrt(2) ** exps)[None, :]


class DTLZ5(DTLZTestSuit):
    def __init__(self, d=None, m=None, ref_num=1000):
        m = 3 if m is None else m
        d = m + 9 if d is None else d
        super().__init__(d, m, ref_num)

    def _objectives(self, Xp, g):
        m = self.m
        temp = g.expand(-1, max(m - 2, 0))
        Xp = torch.cat([Xp[:, :1], (1 + 2 * temp * Xp[:, 1 : m - 1]) / (2 + 2 * temp)], 1)
        return _spherical(Xp, m, g)

    def pf(self):
        return _degenerate_pf(self.ref_num, self.m)


class DTLZ6(DTLZ5):
    _g_partial = staticmethod(lambda Y: (Y**0.1).sum(1))


class DTLZ7(DTLZTestSuit):
    def __init__(self, d=None, m=None, ref_num=1000):
        m = 3 if m is None else m
        d = m + 19 if d is None else d
        super().__init__(d, m, ref_num)
        self.sample = GridSampling(self.ref_num * self.m, self.m - 1)

    _g_partial = staticmethod(lambda Y: Y.sum(1))

    def _g_from(self, S, d):
        return 1 + 9 * S / (d - self.m + 1)

    def _objectives(self, fm, g):
        last = (1 + g) * (self.m - (fm / (1 + g) * (1 + torch.sin(3 * math.pi * fm))).sum(1, keepdim=True))
        return torch.cat([fm, last], 1)

    def pf(self):
        interval = torch.tensor([0, 0.251412, 0.631627, 0.859401])
        median = (interval[1] - interval[0]) / (interval[3] - interval[2] + interval[1] - interval[0])
        x = self.sample()[0]
        x = torch.where(x <= median, x * (interval[1] - interval[0]) / median + interval[0], (x - median) * (interval[3] - interval[2]) / (1 - median) + interval[2])
        last = 2 * (self.m - (x / 2 * (1 + torch.sin(3 * math.pi * x))).sum(1, keepdim=True))
        return torch.cat([x, last], 1)
