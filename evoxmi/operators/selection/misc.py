"""Selection operators: tournament, top-k, roulette wheel, RVEA's APD selection,
uniform random subset, random pbest (reference ``operators/selection/*.py``)."""
from __future__ import annotations

from typing import Callable

import torch

from evoxmi.ops.sort import topk as _topk

from ...ops import random as rnd
from ...utils.common import cos_dist


def move_n_small_numbers(a: torch.Tensor, n):
    """Stable partition that moves the ``n`` smallest elements to the front
    (reference ``crossover/differential_evolution.py:49-60``).  Returns (values, indices)."""
    n = int(n)
    order = torch.argsort(a, stable=True)
    small = torch.zeros(a.shape[0], dtype=torch.bool, device=a.device)
    small[order[:n]] = True
    # stable partition: small ones keep their original relative order
    key = (~small).to(torch.int64) * a.shape[0] + torch.arange(a.shape[0], device=a.device)
    idx = torch.argsort(key)
    return a[idx], idx


def select_rand_pbest(key, percent, population, fitness):
    """Random member of the top ⌊p·N⌋ (reference ``find_pbest.py:12-25``)."""
    n = population.shape[0]
    top = max(int(n * float(percent)), 1)
    _, moved_ids = move_n_small_numbers(fitness, top)
    moved_pop = population[moved_ids]
    random_ids = rnd.choice(key, n, (n,), replace=False).to(population.device)
    moved_random, _ = move_n_small_numbers(random_ids, top)
    return moved_pop[moved_random[0]]


def tournament_single_fit(key, pop, fit, n_round, tournament_func=torch.argmin, tournament_size=2):
    n = fit.shape[0]
    chosen = rnd.randint(key, (n_round, tournament_size), 0, n).to(fit.device)
    cand = fit[chosen]
    win = torch.stack([tournament_func(c) for c in cand]) if tournament_func is not torch.argmin else torch.argmin(cand, dim=1)
    index = chosen[torch.arange(n_round, device=fit.device), win]
    return pop[index], index


def tournament_multi_fit(key, pop, fit, n_round, tournament_func=None, tournament_size=2):
    """Lexicographic winner over the objective columns (first column primary)."""
    n = fit.shape[0]
    chosen = rnd.randint(key, (n_round, tournament_size), 0, n).to(fit.device)
    cand = fit[chosen]  # (R, T, K)
    order = torch.arange(tournament_size, device=fit.device).expand(n_round, -1)
    for col in reversed(range(cand.shape[2])):
        vals = torch.gather(cand[:, :, col], 1, order)
        o = torch.argsort(vals, dim=1, stable=True)
        order = torch.gather(order, 1, o)
    index = chosen[torch.arange(n_round, device=fit.device), order[:, 0]]
    return pop[index], index


class Tournament:
    def __init__(self, n_round: int, tournament_func: Callable = torch.argmin, tournament_size: int = 2, multi_objective: bool = False):
        self.n_round = n_round
        self.tournament_func = tournament_func
        self.tournament_size = tournament_size
        self.multi_obj = multi_objective

    def __call__(self, key, pop, *args):
        if self.multi_obj:
            fit = torch.stack(args, 1) if len(args) > 1 else args[0]
            return tournament_multi_fit(key, pop, fit, self.n_round, self.tournament_func, self.tournament_size)
        return tournament_single_fit(key, pop, args[0], self.n_round, self.tournament_func, self.tournament_size)


def topk_fit(population, fitness, topk):
    v, i = _topk(fitness, topk, largest=False)
    return population[i], v


class TopkFit:
    def __init__(self, topk):
        self.topk = topk

    def __call__(self, population, fitness):
        return topk_fit(population, fitness, self.topk)


class RouletteWheelSelection:
    """Smaller fitness ⇒ larger selection probability (reference ``roulette_wheel.py``)."""

    def __init__(self, n):
        self.n = n

    def __call__(self, key, x, fitness):
        f = fitness - torch.clamp(fitness.min(), max=0) + 1e-6
        c = torch.cumsum(1.0 / f, 0)
        c = c / c.max()
        u = rnd.uniform(key, (self.n,)).to(x.device)
        idx = torch.searchsorted(c, u).clamp_max(x.shape[0] - 1)
        return x[idx], idx


def ref_vec_guided(x, f, v, theta):
    """RVEA angle-penalised distance selection (reference ``rvea_selection.py:9-54``).
    Rows of ``x``/``f`` may be NaN padding; empty reference vectors yield NaN rows."""
    n, m = f.shape
    nv = v.shape[0]
    obj = f - torch.nan_to_num(f, nan=float("inf")).min(0).values
    obj = torch.clamp(obj, min=1e-32)
    cosine = cos_dist(v, v)
    cosine = cosine.masked_fill(torch.eye(nv, dtype=torch.bool, device=v.device), 0)
    cosine = cosine.clamp(0, 1)
    gamma = torch.arccos(cosine).min(1).values
    angle = torch.arccos(cos_dist(torch.nan_to_num(obj, nan=0.0), v).clamp(0, 1))
    nan_mask = torch.isnan(obj).any(1)
    associate = torch.argmin(angle, 1)
    associate = torch.where(nan_mask, torch.full_like(associate, -1), associate)
    norm = torch.sqrt((torch.nan_to_num(obj, nan=0.0) ** 2).sum(1))
    member = associate[:, None] == torch.arange(nv, device=v.device)[None, :]  # (n, nv)
    apd = (1 + m * theta * angle / gamma[None, :]) * norm[:, None]
    apd = torch.where(member, apd, torch.full_like(apd, float("inf")))
    next_ind = torch.argmin(apd, 0)
    empty = ~member.any(0)
    nan_row = torch.full((1,), float("nan"), device=x.device, dtype=x.dtype)
    next_x = torch.where(empty[:, None], nan_row, x[next_ind])
    next_f = torch.where(empty[:, None], nan_row, f[next_ind])
    return next_x, next_f


class ReferenceVectorGuided:
    def __call__(self, x, f, v, theta):
        return ref_vec_guided(x, f, v, theta)


def uniform_rand(key, pop, *others, prob):
    num = int(pop.shape[0] * prob)
    chosen = rnd.randint(key, (num,), 0, pop.shape[0]).to(pop.device)
    if not others:
        return pop[chosen]
    return (pop[chosen], *[o[chosen] for o in others])


class UniformRand:
    def __init__(self, prob):
        self.prob = prob

    def __call__(self, key, pop, *others):
        return uniform_rand(key, pop, *others, prob=self.prob)
