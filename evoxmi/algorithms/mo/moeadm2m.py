"""MOEA/D-M2M (Liu, Gu & Zhang 2014; reference ``algorithms/mo/moeadm2m.py:96-203``).

The objective space is split into K sub-regions by K direction vectors; each keeps S
members chosen by NSGA-II ranking among the solutions associated with it (padded
with random solutions when fewer are available).  Variation is the M2M
crossover/mutation whose spread shrinks with ``gen / max_gen``.  The per-region
selection of the reference (a ``fori_loop`` over regions each running its own
non-dominated sort) is done for all regions at once: the sort of region k only
involves its own members, so one non-dominated sort of the merged set restricted
by region gives identical ranks (dominance is evaluated within the region mask).
"""
from __future__ import annotations

import torch

from ...core import State
from ...operators.sampling import UniformSampling
from ...operators.selection.non_dominate import crowding_distance, lexsort
from ...ops import random as rnd
from ...utils.common import cos_dist, dominate_relation
from .common import MOAlgorithm


def m2m_crossover(key, p1, p2, scale):
    n, d = p1.shape
    k1, k2 = rnd.split(key)
    rc = (2 * rnd.uniform(k1, (n, 1)).to(p1.device) - 1) * (1 - rnd.uniform(k2, (n, 1)).to(p1.device)) ** (-((1 - scale) ** 0.7))
    return p1 + rc * (p1 - p2)


def m2m_mutation(key, p1, off, scale, lb, ub):
    n, d = p1.shape
    k1, k2, k3, k4 = rnd.split(key, 4)
    u = lambda k: rnd.uniform(k, (n, d)).to(p1.device)
    rm = 0.25 * (2 * u(k1) - 1) * (1 - u(k2)) ** (-((1 - scale) ** 0.7))
    site = u(k3) < (1 / d)
    off = torch.where(site, off + rm * (ub - lb), off)
    r = u(k4)
    off = torch.where(off < lb, lb + 0.5 * r * (p1 - lb), off)
    return torch.where(off > ub, ub - 0.5 * r * (ub - p1), off)


def _rank_within(obj, region):
    """Non-dominated rank of every point among the points of its own region."""
    n = obj.shape[0]
    dom = dominate_relation(obj, obj) & (region[:, None] == region[None, :])
    rank = torch.zeros(n, dtype=torch.int64, device=obj.device)
    remaining = torch.ones(n, dtype=torch.bool, device=obj.device)
    r = 0
    while bool(remaining.any()):
        cnt = (dom & remaining[:, None]).sum(0)
        front = remaining & (cnt == 0)
        rank[front] = r
        remaining &= ~front
        r += 1
    return rank


def associate(key, pop, obj, w, s):
    k = w.shape[0]
    n = pop.shape[0]
    region = torch.argmax(cos_dist(obj, w), 1)
    rank = _rank_within(obj, region).to(torch.float32)
    cols = []
    rad = rnd.randint(key, (s,), 0, n).to(pop.device)
    for i in range(k):
        mask = region == i
        cnt = int(mask.sum())
        if cnt < s:
            members = torch.nonzero(mask).flatten()
            cols.append(torch.cat([members, rad[cnt:]]))
        else:
            rk = torch.where(mask, rank, torch.full_like(rank, float("inf")))
            order = torch.argsort(rk, stable=True)
            worst = rk[order[s - 1]]
            cd = crowding_distance(obj, rk == worst)
            cols.append(lexsort([-cd, rk])[:s])
    part = torch.stack(cols, 1).T.reshape(-1)  # region-major (Fortran flatten of (s, k))
    return pop[part], obj[part]


class MOEADM2M(MOAlgorithm):
    def __init__(self, lb, ub, n_objs, pop_size, k=10, max_gen=100, mutation_op=None, crossover_op=None, seed=0):
        super().__init__(lb, ub, n_objs, pop_size)
        self.max_gen = max_gen
        w, kk = UniformSampling(k, n_objs)()
        self.w = w.to(lb.device)
        self.k = int(kk)
        self.pop_size = int(-(-pop_size // self.k) * self.k)
        self.s = self.pop_size // self.k

    def setup(self, key):
        return super().setup(key).update(gen=torch.zeros((), dtype=torch.int64, device=self.lb.device))

    def ask(self, state):
        key, k_loc, k_glob, k_rnd, x_key, mut_key = rnd.split(state.key, 6)
        dev = state.population.device
        s, k, N = self.s, self.k, self.pop_size
        scale = state.gen.to(torch.float32) / self.max_gen
        local = rnd.randint(k_loc, (s, k), 0, s).to(dev) + torch.arange(0, s * k, s, device=dev)[None, :]
        glob = rnd.randint(k_glob, (N,), 0, N).to(dev)
        pool = torch.where(rnd.uniform(k_rnd, (s, k)).to(dev).reshape(-1) < 0.7, glob, local.reshape(-1))
        off = m2m_crossover(x_key, state.population, state.population[pool], scale)
        off = m2m_mutation(mut_key, state.population, off, scale, self.lb, self.ub)
        return off, state.update(next_generation=off, key=key, gen=state.gen + 1)

    def init_tell(self, state, fitness):
        key, sub = rnd.split(state.key)
        pop, obj = associate(sub, state.population, fitness, self.w, self.s)
        return state.update(population=pop, fitness=obj, key=key)

    def tell(self, state, fitness):
        key, sub = rnd.split(state.key)
        pop, obj = associate(sub, torch.cat([state.population, state.next_generation]), torch.cat([state.fitness, fitness]), self.w, self.s)
        return state.update(population=pop, fitness=obj, key=key)
