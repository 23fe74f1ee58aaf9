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

    _funcs = (sphere_func,)
    _cosine = False
    # decision-axis sharding (evoxmi.parallel.dim_sharded): full rows (the linkage needs
    # x₁), each rank reduces the parts of the m·nk variable groups inside its column block
    dim_shard_full_rows = True
    dim_halo = 0
    dim_shard_max_terms = True  # the Schwefel groups reduce with max

    def setup(self, key):
        return State(key=key)

    def pf(self):
        return UniformSampling(self.ref_num * self.m, self.m)()[0] / 2

    def _groups(self):
        """(objective k, column start, length, inner function) of every subcomponent."""
        out = []
        for k, (len_, sublen, func) in enumerate(zip(self.len, self.sublen, cycle(self._funcs))):
            if k >= self.m:
                break
            for j in range(self.nk):
                out.append((k, len_ + self.m - 1 + j * sublen, sublen, func))
        return out

    def partial_terms(self, X, col0, d, own):
        n, m = X.shape[0], self.m
        c1 = col0 + own
        x = self._link(X, self._cosine)
        groups = self._groups()
        T = X.new_zeros(n, 3 * len(groups) + m - 1)
        Tm = X.new_zeros(n, len(groups))
        for gi, (k, s, L, func) in enumerate(groups):
            a, b = max(s, col0), min(s + L, c1)
            if a >= b:
                continue
            z = x[:, a:b]
            if func is sphere_func:
                T[:, 3 * gi] = (z * z).sum(1)
            elif func is _rastrigin:
                T[:, 3 * gi] = (z * z - 10 * torch.cos(2 * math.pi * z) + 10).sum(1)
            elif func is rosenbrock_func:
                hi = min(b, s + L - 1)  # pairs (i, i + 1) inside the group whose left index is owned
                if hi > a:
                    u, v = x[:, a:hi], x[:, a + 1 : hi + 1]
                    T[:, 3 * gi] = (100 * (v - u * u) ** 2 + (u - 1) ** 2).sum(1)
            elif func is griewank_func:
                i = torch.arange(a - s + 1, b - s + 1, device=X.device, dtype=X.dtype)
                cz = torch.cos(z / torch.sqrt(i))
                T[:, 3 * gi] = (z * z).sum(1) / 4000
                T[:, 3 * gi + 1] = torch.log(torch.abs(cz)).sum(1)
                T[:, 3 * gi + 2] = (cz < 0).to(X.dtype).sum(1)
            elif func is _ackley:
                T[:, 3 * gi] = (z * z).sum(1)
                T[:, 3 * gi + 1] = torch.cos(2 * math.pi * z).sum(1)
            elif func is _schwefel:
                Tm[:, gi] = torch.abs(z).amax(1)
        lo, hi = col0, min(c1, m - 1)
        if hi > lo:  # the position variables x₁…x_{m−1} for the front
            T[:, 3 * len(groups) + lo : 3 * len(groups) + hi] = X[:, lo:hi]
        return T, Tm

    def combine_terms(self, T, d):
        T, Tm = T
        n, m = T.shape[0], self.m
        groups = self._groups()
        g = T.new_zeros(n, m)
        for gi, (k, s, L, func) in enumerate(groups):
            t0, t1, t2 = T[:, 3 * gi], T[:, 3 * gi + 1], T[:, 3 * gi + 2]
            if func is griewank_func:
                sign = 1 - 2 * torch.remainder(torch.round(t2), 2)
                v = t0 - sign * torch.exp(t1) + 1
            elif func is _ackley:
                v = -20 * torch.exp(-0.2 * torch.sqrt(t0 / L)) - torch.exp(t1 / L) + 20 + math.e
            elif func is _schwefel:
                v = Tm[:, gi]
            else:
                v = t0
            g[:, k] = g[:, k] + v / (L * self.nk)
        Xf = T[:, 3 * len(groups) :]
        return self._finish(Xf, g)

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


class _Linear(LSMOP):
    def evaluate(self, state, X):
        return self._finish(X, self._g(self._funcs, X, self._cosine)), state

    def _finish(self, X, g):
        return self._linear_front(X, g)


class LSMOP1(_Linear):
    _funcs = (sphere_func,)


class LSMOP2(_Linear):
    _funcs = (griewank_func, _schwefel)


class LSMOP3(_Linear):
    _late_d = False
    _funcs = (_rastrigin, rosenbrock_func)


class LSMOP4(_Linear):
    _funcs = (_ackley, griewank_func)


class _SphericalPF:
    def pf(self):
        f = UniformSampling(self.ref_num * self.m, self.m)()[0] / 2
        return f / torch.sqrt((f * f).sum(1, keepdim=True))


class _Spherical(LSMOP):
    _cosine = True

    def evaluate(self, state, X):
        return self._finish(X, self._g(self._funcs, X, self._cosine)), state

    def _finish(self, X, g):
        return self._spherical_front(X, g)


class LSMOP5(_SphericalPF, _Spherical):
    _funcs = (sphere_func,)


class LSMOP6(_Spherical):
    _funcs = (rosenbrock_func, _schwefel)


class LSMOP7(_SphericalPF, _Spherical):
    _funcs = (_ackley, rosenbrock_func)


class LSMOP8(_SphericalPF, _Spherical):
    _funcs = (griewank_func, sphere_func)


class LSMOP9(LSMOP):
    _funcs = (sphere_func, _ackley)
    _cosine = True

    def evaluate(self, state, X):
        return self._finish(X, self._g(self._funcs, X, self._cosine)), state

    def _finish(self, X, g):
        m = self.m
        g = 1 + g.sum(1, keepdim=True)
        fm = X[:, : m - 1]
        last = (1 + g) * (m - (fm / (1 + g) * (1 + torch.sin(3 * math.pi * fm))).sum(1, keepdim=True))
        return torch.cat([fm, last], 1)

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
