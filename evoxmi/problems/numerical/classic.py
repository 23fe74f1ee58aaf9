"""Classic single-objective benchmark functions (K5 of SURVEY §2.10).

Reference: ``problems/numerical/{ackley,griewank,rastrigin,rosenbrock,schwefel,sphere}.py``.
Each is a fused elementwise + row reduction.  On a GPU the whole (N, d) → (N,)
evaluation is one HIP launch (``csrc/kernels/classic.hip``: one wave64 per row,
16-byte loads, wave-shuffle reduction); on CPU the torch expressions below are
both the implementation and the numerics oracle.  The ``*_func(X)`` forms are
reused by LSMOP.
"""
from __future__ import annotations

import math

import torch

from ...core import Problem
from ...ops import numerical as _nops

FUNC_IDS = {"sphere": 0, "ackley": 1, "rastrigin": 2, "rosenbrock": 3, "griewank": 4, "schwefel": 5, "ellipsoid": 6}


def _dispatch(name, X, a=0.0, b=0.0, c=0.0):
    if X.is_cuda and X.dtype == torch.float32:
        return _nops.classic_eval(X, FUNC_IDS[name], a, b, c)
    return None


def sphere_func(X):
    r = _dispatch("sphere", X)
    return r if r is not None else (X * X).sum(-1)


def ackley_func(a, b, c, X):
    r = _dispatch("ackley", X, a, b, c)
    if r is not None:
        return r
    return -a * torch.exp(-b * torch.sqrt((X * X).mean(-1))) - torch.exp(torch.cos(c * X).mean(-1)) + a + math.e


def rastrigin_func(X):
    r = _dispatch("rastrigin", X)
    if r is not None:
        return r
    return 10 * X.shape[-1] + (X * X - 10 * torch.cos(2 * math.pi * X)).sum(-1)


def rosenbrock_func(X):
    r = _dispatch("rosenbrock", X)
    if r is not None:
        return r
    return (100 * (X[..., 1:] - X[..., :-1] ** 2) ** 2 + (X[..., :-1] - 1) ** 2).sum(-1)


def griewank_func(X):
    r = _dispatch("griewank", X)
    if r is not None:
        return r
    i = torch.arange(1, X.shape[-1] + 1, device=X.device, dtype=X.dtype)
    return (X * X).sum(-1) / 4000 - torch.prod(torch.cos(X / torch.sqrt(i)), -1) + 1


def schwefel_func(X):
    r = _dispatch("schwefel", X)
    if r is not None:
        return r
    return 418.9828872724338 * X.shape[-1] - (X * torch.sin(torch.sqrt(torch.abs(X)))).sum(-1)


def ellipsoid_func(X):
    r = _dispatch("ellipsoid", X)
    if r is not None:
        return r
    i = torch.arange(1, X.shape[-1] + 1, device=X.device, dtype=X.dtype)
    return (i * X * X).sum(-1)


# ---------------------------------------------------------------------------
# Decision-axis sharding protocol (SURVEY §2.2 strategy P2, used by
# evoxmi.parallel.DimShardedProblem): ``partial_terms(Xb, col0, d, own)`` maps the
# column block ``Xb`` (its first ``own`` columns start at global column ``col0``;
# ``dim_halo`` extra columns follow) to per-row additive terms (N, k); the terms of
# all blocks are summed by one all-reduce and ``combine_terms(T, d)`` finishes.


class Sphere(Problem):
    dim_halo = 0

    def evaluate(self, state, X):
        return sphere_func(X), state

    def partial_terms(self, Xb, col0, d, own):
        return (Xb * Xb).sum(-1, keepdim=True)

    def combine_terms(self, T, d):
        return T[:, 0]


class Ackley(Problem):
    def __init__(self, a=20.0, b=0.2, c=2 * math.pi):
        super().__init__()
        self.a, self.b, self.c = float(a), float(b), float(c)

    dim_halo = 0

    def evaluate(self, state, X):
        return ackley_func(self.a, self.b, self.c, X), state

    def partial_terms(self, Xb, col0, d, own):
        return torch.stack([(Xb * Xb).sum(-1), torch.cos(self.c * Xb).sum(-1)], -1)

    def combine_terms(self, T, d):
        return -self.a * torch.exp(-self.b * torch.sqrt(T[:, 0] / d)) - torch.exp(T[:, 1] / d) + self.a + math.e


class Rastrigin(Problem):
    dim_halo = 0

    def evaluate(self, state, X):
        return rastrigin_func(X), state

    def partial_terms(self, Xb, col0, d, own):
        return (Xb * Xb - 10 * torch.cos(2 * math.pi * Xb)).sum(-1, keepdim=True)

    def combine_terms(self, T, d):
        return 10 * d + T[:, 0]


class Rosenbrock(Problem):
    dim_halo = 1  # the term of column i needs x_{i+1}

    def evaluate(self, state, X):
        return rosenbrock_func(X), state

    def partial_terms(self, Xb, col0, d, own):
        n = min(own, d - 1 - col0)  # pair terms whose left column is owned here
        if n <= 0:
            return Xb.new_zeros(Xb.shape[0], 1)
        a, b = Xb[:, :n], Xb[:, 1 : n + 1]
        return (100 * (b - a * a) ** 2 + (a - 1) ** 2).sum(-1, keepdim=True)

    def combine_terms(self, T, d):
        return T[:, 0]


class Griewank(Problem):
    dim_halo = 0

    def evaluate(self, state, X):
        return griewank_func(X), state

    def partial_terms(self, Xb, col0, d, own):
        # the product is carried as (Σ log|cos|, #negative factors) so it stays additive
        i = torch.arange(col0 + 1, col0 + Xb.shape[1] + 1, device=Xb.device, dtype=Xb.dtype)
        cs = torch.cos(Xb / torch.sqrt(i))
        return torch.stack([(Xb * Xb).sum(-1), torch.log(cs.abs()).sum(-1), (cs < 0).sum(-1).to(Xb.dtype)], -1)

    def combine_terms(self, T, d):
        sign = 1 - 2 * torch.remainder(T[:, 2], 2)
        return T[:, 0] / 4000 - sign * torch.exp(T[:, 1]) + 1


class Schwefel(Problem):
    """Minimum at x = [420.9687462275036, ...]."""

    dim_halo = 0

    def evaluate(self, state, X):
        return schwefel_func(X), state

    def partial_terms(self, Xb, col0, d, own):
        return (Xb * torch.sin(torch.sqrt(torch.abs(Xb)))).sum(-1, keepdim=True)

    def combine_terms(self, T, d):
        return 418.9828872724338 * d - T[:, 0]


class Ellipsoid(Problem):
    dim_halo = 0

    def evaluate(self, state, X):
        return ellipsoid_func(X), state

    def partial_terms(self, Xb, col0, d, own):
        i = torch.arange(col0 + 1, col0 + Xb.shape[1] + 1, device=Xb.device, dtype=Xb.dtype)
        return (i * Xb * Xb).sum(-1, keepdim=True)

    def combine_terms(self, T, d):
        return T[:, 0]
