"""LSMOP1–9 large-scale multi-objective problems (Cheng et al. 2017; reference
``problems/numerical/lsmop.py:18-455``).

nk = 5 subcomponents per objective with chaotic group sizes
``c_i = 3.8·c_{i−1}(1 − c_{i−1})`` (c_0 = 3.8·0.1·0.9); the linkage transform
``x_j ← (1 + t_j)·x_j − 10·x_1`` (t_j = j/d for LSMOP1–4, cos(π j /(2d)) for
LSMOP5–9) followed by grouped inner functions (sphere / Griewank / Rosenbrock /
Ackley / Schwefel-max / Rastrigin).  Quirk kept: when
``d is None`` most classes compute the groups with d = 100·m and then set
``self.d = m + 4``.  The group reduction is a segmented row sum (one pass per
group on the (n, d) matrix).
"""
from __future__ import annotations

import math
from itertools import cycle

import torch

from ...core import Problem, State
from ...operators.sampling import UniformSampling
from .classic import ackley_func, griewank_func, rosenbrock_func, sphere_func


def _schwefel(X):
    return torch.abs(X).amax(-1)


def _rastrigin(X):
    return (X**2 - 10 * torch.cos(2 * math.pi * X) + 10).sum(1)


def _ackley(X):
    return ackley_func(20.0, 0.2, 2 * math.pi, X)


_FUNC_ID = {sphere_func: 0, griewank_func: 1, rosenbrock_func: 2, _ackley: 3, _schwefel: 4, _rastrigin: 5}


class LSMOP(Problem):
    _late_d = True  # groups computed with d = 100·m when d is None, then d = m + 4

    def __init__(self, d=None, m=None, ref_num=1000):
        super().__init__()
        self.nk = 5
        self.m = 3 if m is None else m
        d_groups = self.m * 100 if d is None else d
        if not self._late_d:
            d_groups = self.m + 4 if d is None else d
        self.ref_num = ref_num
        c = [3.8 * 0.1 * (1 - 0.1)]
        for _ in range(1, self.m):
            c.append(3.8 * c[-1] * (1 - c[-1]))
        csum = sum(c)
        self.sublen = tuple(int(math.floor(ci / csum * d_groups / self.nk)) for ci in c)
        lens = [0]
        for s in self.sublen:
            lens.append(lens[-1] + s * self.nk)
        self.len = tuple(lens)
        self.d = self.m + 4 if d is None else d

    def setup(self, key):
        return State(key=key)

    def pf(self):
        return UniformSampling(self.ref_num * self.m, self.m)()[0] / 2

    def _g(self, inner_funcs, X, cosine: bool):
        """Distance terms g (n, m) from the RAW decisions: on a GPU one fused pass
        (``mo_problems.hip: lsmop_g_kernel``), else link + grouped reductions."""
        if X.is_cuda and X.dtype == torch.float32 and 2 <= self.m <= 16 and self.len[self.m] + self.m - 1 <= X.shape[1]:
            from ...ops import _ext

            funcs = [_FUNC_ID[f] for _, f in zip(range(self.m), cycle(inner_funcs))]
            starts = [self.len[k] + self.m - 1 for k in range(self.m)]
            return _ext.ops().lsmop_g(X.contiguous(), starts, list(self.sublen), funcs, self.nk, int(cosine))
        return self._calc_g(inner_funcs, self._link(X, cosine))

    def _calc_g(self, inner_funcs, x):
        n = x.shape[0]
        gs = []
        for len_, sublen, func in zip(self.len, self.sublen, cycle(inner_funcs)):
            acc = torch.zeros(n, dtype=x.dtype, device=x.device)
            for j in range(self.nk):
                start = len_ + self.m - 1 + j * sublen
                acc = acc + func(x[:, start : start + sublen].contiguous())
            gs.append(acc / (sublen * self.nk))  # host scalar: no H2D copy (graph-capturable)
        return torch.stack(gs, 1)

    def _link(self, X, cosine: bool):
        n, d = X.shape
        m = self.m
        j = torch.arange(m, d + 1, dtype=X.dtype, device=X.device) / d
        t = torch.cos(j * math.pi / 2) if cosine else j
        tail = (1 + t)[None, :] * X[:, m - 1 :] - X[:, :1] * 10
        return torch.cat([X[:, : m - 1], tail], 1)

    def _linear_front(self, X, g):
        n, m = X.shape[0], self.m
        ones = torch.ones((n, 1), dtype=X.dtype, device=X.device)
        a = torch.flip(torch.cumprod(torch.cat([ones, X[:, : m - 1]], 1), 1), [1])
        b = torch.cat([ones, 1 - torch.flip(X[:, : m - 1], [1])], 1)
        return (1 + g) * a * b

    def _spherical_front(self, X, g):
        n, m = X.shape[0], self.m
        ones = torch.ones((n, 1), dtype=X.dtype, device=X.device)
        g2 = 1 + g + torch.cat([g[:, 1:], torch.zeros((n, 1), dtype=X.dtype, device=X.device)], 1)
        a = torch.flip(torch.cumprod(torch.cat([ones, torch.cos(X[:, : m - 1] * math.pi / 2)], 1), 1), [1])
        b = torch.cat([ones, torch.sin(torch.flip(X[:, : m - 1], [1]) * math.pi / 2)], 1)
        return g2 * a * b


class LSMOP1(LSMOP):
    def evaluate(self, state, X):
        return self._linear_front(X, self._g([sphere_func], X, False)), state


class LSMOP2(LSMOP):
    def evaluate(self, state, X):
        return self._linear_front(X, self._g([griewank_func, _schwefel], X, False)), state


class LSMOP3(LSMOP):
    _late_d = False

    def evaluate(self, state, X):
        return self._linear_front(X, self._g([_rastrigin, rosenbrock_func], X, False)), state


class LSMOP4(LSMOP):
    def evaluate(self, state, X):
        return self._linear_front(X, self._g([_ackley, griewank_func], X, False)), state


class _SphericalPF:
    def pf(self):
        f = UniformSampling(self.ref_num * self.m, self.m)()[0] / 2
        return f / torch.sqrt((f * f).sum(1, keepdim=True))


class LSMOP5(_SphericalPF, LSMOP):
    def evaluate(self, state, X):
        return self._spherical_front(X, self._g([sphere_func], X, True)), state


class LSMOP6(LSMOP):
    def evaluate(self, state, X):
        return self._spherical_front(X, self._g([rosenbrock_func, _schwefel], X, True)), state


class LSMOP7(_SphericalPF, LSMOP):
    def evaluate(self, state, X):
        return self._spherical_front(X, self._g([_ackley, rosenbrock_func], X, True)), state


class LSMOP8(_SphericalPF, LSMOP):
    def evaluate(self, state, X):
        return self._spherical_front(X, self._g([griewank_func, sphere_func], X, True)), state


class LSMOP9(LSMOP):
    def evaluate(self, state, X):
        m = self.m
        g = 1 + self._g([sphere_func, _ackley], X, True).sum(1, keepdim=True)
        fm = X[:, : m - 1]
        last = (1 + g) * (m - (fm / (1 + g) * (1 + torch.sin(3 * math.pi * fm))).sum(1, keepdim=True))
        return torch.cat([fm, last], 1), state

    def pf(self):
        interval = [0, 0.251412, 0.631627, 0.859401]
        median = (interval[1] - interval[0]) / (interval[3] - interval[2] + interval[1] - interval[0])
        N = self.ref_num * self.m
        M = self.m - 1
        gap = torch.linspace(0, 1, int(math.ceil(N ** (1 / M))))
        c = torch.meshgrid(*([gap] * M), indexing="xy")
        X = torch.stack([x.reshape(-1) for x in c], 1)
        X = torch.where(X <= median, X * (interval[1] - interval[0]) / median + interval[0], (X - median) * (interval[3] - interval[2]) / (1 - median) + interval[2])
        return torch.cat([X, 2 * (self.m - (X / 2 * (1 + torch.sin(3 * math.pi * X))).sum(1, keepdim=True))], 1)
