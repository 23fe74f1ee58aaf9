"""Differential-evolution operators (reference ``operators/crossover/differential_evolution.py``),
including the fork's ``de_diff_sum*`` family and bin/exp/arith crossovers.

Each reference function works on one individual and is ``vmap``-ed by the
algorithms; here every operator has a **batched** form (all N trial vectors in
one call, ``batched_*``) which is what the algorithms use, plus the single-row
form for API parity.  Semantics follow the reference including its quirks
(indices equal to the target are remapped to ``pop_size_reduced − 1``; the
exponential crossover length is ``min(Geometric(CR), d) − 1``).
"""
from __future__ import annotations

import math

import torch

from evoxmi.ops.sort import topk as _topk

from ...ops import random as rnd


def _de_mutation(x1, x2, x3, F):
    return x1 + F * (x2 - x3)


def _de_crossover(key, new_x, x, CR):
    mask = rnd.uniform(key, x.shape).to(x.device) < CR
    return torch.where(mask, new_x, x)


def differential_evolve(key, x1, x2, x3, F, CR):
    _, de_key = rnd.split(key)
    return _de_crossover(de_key, _de_mutation(x1, x2, x3, F), x1, CR)


class DifferentialEvolve:
    def __init__(self, F=0.5, CR=1):
        self.F, self.CR = F, CR

    def __call__(self, key, p1, p2, p3):
        return differential_evolve(key, p1, p2, p3, self.F, self.CR)


def move_n_small_numbers(array: torch.Tensor, n):
    """Stable partition moving every element ≤ the n-th smallest to the front."""
    n = int(n)
    nth = torch.sort(array).values[n - 1]
    cond = (array > nth).to(torch.int64)
    idx = torch.argsort(cond, stable=True)
    return array[idx], idx


def _distinct_rows(key, rows: int, k: int, upper, device):
    """``rows`` independent samples of ``k`` distinct integers from [0, upper)."""
    upper = int(upper)
    u = rnd.uniform(key, (rows, upper)).to(device)
    return torch.argsort(u, dim=1, stable=True)[:, :k]


def _signed_sum(members: torch.Tensor, nd) -> torch.Tensor:
    """members: (N, P, d) with P = diff_padding_num; Σ_{j=1..2nd} (−1)^{j+1} x_j, zero beyond 2nd."""
    N, P, d = members.shape
    j = torch.arange(P, device=members.device)
    nd = torch.as_tensor(nd, device=members.device).reshape(-1, 1) if not isinstance(nd, int) else torch.full((N, 1), nd, device=members.device)
    keep = (j[None, :] >= 1) & (j[None, :] < 2 * nd + 1)
    sign = torch.where(j % 2 == 1, 1.0, -1.0).to(members.dtype)
    coef = keep.to(members.dtype) * sign[None, :]
    return torch.einsum("np,npd->nd", coef, members)


def batched_de_diff_sum(key, diff_padding_num: int, num_diff_vects, population, pop_size_reduced=None):
    """Difference-vector sums and base indices for all N individuals.

    Returns ``(difference_sum (N, d), rand_vect_idx (N,))``.
    """
    N, d = population.shape
    P = N if pop_size_reduced is None else int(pop_size_reduced)
    choice = _distinct_rows(key, N, diff_padding_num, P, population.device)
    index = torch.arange(N, device=population.device)[:, None]
    choice = torch.where(choice == index, torch.full_like(choice, P - 1), choice)
    members = population[choice]
    return _signed_sum(members, num_diff_vects), choice[:, 0]


def de_diff_sum(key, diff_padding_num, num_diff_vects, index, population, pop_size_reduced=None, replace=False):
    """Single-individual form (reference ``:63-96``)."""
    N, d = population.shape
    P = N if pop_size_reduced is None else int(pop_size_reduced)
    choice = _distinct_rows(key, 1, diff_padding_num, P, population.device)[0]
    choice = torch.where(choice == int(index), torch.full_like(choice, P - 1), choice)
    s = _signed_sum(population[choice][None], num_diff_vects)[0]
    return s, choice[0]


def batched_de_diff_sum_archive(key, diff_padding_num: int, num_diff_vects, population, archive, pop_size_reduced=None):
    """JADE/SHADE: subtrahends at even positions (≥2) drawn from P ∪ A (NaN archive rows excluded)."""
    N, d = population.shape
    P = N if pop_size_reduced is None else int(pop_size_reduced)
    pa = torch.cat([population, archive], 0)
    nan_rows = torch.isnan(pa.sum(1))
    order = torch.argsort(nan_rows.to(torch.int64), stable=True)  # valid rows first
    pa_moved = pa[order]
    n_valid = (~nan_rows).sum()
    k1, k2 = rnd.split(key)
    base = _distinct_rows(k1, N, diff_padding_num, P, population.device)
    # subtrahend candidates from the valid part of P∪A (at most 2·P rows, reference :121-124)
    upper = 2 * P
    sub = _distinct_rows(k2, N, diff_padding_num, upper, population.device)
    sub = torch.minimum(sub, (n_valid - 1).clamp_min(0).to(sub.dtype))
    j = torch.arange(diff_padding_num, device=population.device)
    even = (j >= 2) & (j % 2 == 0)
    ids = torch.where(even[None, :], sub, base)
    index = torch.arange(N, device=population.device)[:, None]
    ids = torch.where(ids == index, torch.full_like(ids, P - 1), ids)
    members = pa_moved[ids]
    return _signed_sum(members, num_diff_vects), ids[:, 0]


def de_diff_sum_archive(key, diff_padding_num, num_diff_vects, index, population, archive, pop_size_reduced=None, replace=False):
    s, r = batched_de_diff_sum_archive(key, diff_padding_num, num_diff_vects, population, archive, pop_size_reduced)
    i = int(index)
    return s[i], r[i]


def batched_de_diff_sum_rank(key, diff_padding_num: int, num_diff_vects, population, k_factor, fitness, pop_size_reduced=None):
    """LSHADE-RSP rank-based selective pressure: P(i) ∝ k·(N − rank_i) + 1 on the top
    ``pop_size_reduced`` ranks (reference ``:152-194``), without replacement per row."""
    N, d = population.shape
    P = N if pop_size_reduced is None else int(pop_size_reduced)
    ranks = torch.argsort(torch.argsort(fitness, stable=True), stable=True)
    w = k_factor * (N - ranks).to(torch.float32) + 1
    nth = torch.sort(w).values[N - P]
    w = torch.where(w < nth, torch.zeros_like(w), w)
    logp = torch.log(w / w.sum())
    g = rnd.gumbel(key, (N, N)).to(population.device) + logp[None, :]
    choice = _topk(g, diff_padding_num, dim=1)[1]
    index = torch.arange(N, device=population.device)[:, None]
    choice = torch.where(choice == index, torch.full_like(choice, P - 1), choice)
    return _signed_sum(population[choice], num_diff_vects), choice[:, 0]


def de_diff_sum_rank(key, diff_padding_num, num_diff_vects, index, population, k_factor, fitness, pop_size_reduced=None, replace=False):
    s, r = batched_de_diff_sum_rank(key, diff_padding_num, num_diff_vects, population, k_factor, fitness, pop_size_reduced)
    i = int(index)
    return s[i], r[i]


def batched_de_bin_cross(key, mutation, current, CR):
    """Binomial crossover with a forced j_rand per row; CR may be per-row (N,)."""
    N, d = current.shape
    k1, k2 = rnd.split(key)
    jrand = rnd.randint(k1, (N,), 0, d).to(current.device)
    CR = torch.as_tensor(CR, dtype=current.dtype, device=current.device)
    CR = CR.reshape(-1, 1) if CR.ndim else CR
    mask = rnd.uniform(k2, (N, d)).to(current.device) < CR
    mask[torch.arange(N, device=current.device), jrand] = True
    return torch.where(mask, mutation, current)


def de_bin_cross(key, mutation_vector, current_vect, CR):
    return batched_de_bin_cross(key, mutation_vector[None], current_vect[None], CR)[0]


def batched_de_exp_cross(key, mutation, current, CR):
    """Exponential crossover: a window of length min(Geometric(CR), d) − 1 starting at a random n."""
    N, d = current.shape
    k1, k2 = rnd.split(key)
    n = rnd.randint(k1, (N,), 0, d).to(current.device)
    CR = torch.as_tensor(CR, dtype=torch.float32, device=current.device).reshape(-1) * torch.ones(N, device=current.device)
    u = rnd.uniform(k2, (N,)).to(current.device)
    # Geometric(p) on {1, 2, ...}: ceil(log(u) / log(1 − p)); p = 1 ⇒ 1
    geo = torch.where(CR >= 1, torch.ones_like(u), torch.ceil(torch.log(u) / torch.log1p(-CR.clamp(max=1 - 1e-7))))
    L = torch.minimum(geo, torch.full_like(geo, d)) - 1
    j = torch.arange(d, device=current.device)[None, :]
    pos = (j - n[:, None]) % d
    mask = pos < L[:, None]
    return torch.where(mask, mutation, current)


def de_exp_cross(key, mutation_vector, current_vect, CR):
    return batched_de_exp_cross(key, mutation_vector[None], current_vect[None], CR)[0]


def de_arith_recom(mutation_vector, current_vect, K):
    K = torch.as_tensor(K, dtype=current_vect.dtype, device=current_vect.device)
    if K.ndim == 1 and current_vect.ndim == 2:
        K = K[:, None]
    return current_vect + K * (mutation_vector - current_vect)


batched_de_arith_recom = de_arith_recom
