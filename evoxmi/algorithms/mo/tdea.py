"""θ-DEA (Yuan et al. 2016; reference ``algorithms/mo/tdea.py:100-178``).

NSGA-III-style normalisation (ideal point, hyperplane through extreme points with
fallback to the worst point), clustering to the closest reference direction and
θ-non-dominated sorting (rank inside each cluster by d1 + θ·d2, θ = 5, 10⁶ on the
axes).  The per-cluster ranking loop of the reference is one (cluster, value) sort.
"""
from __future__ import annotations

import torch

from ...core import State
from ...operators.sampling import UniformSampling
from ...operators.selection.non_dominate import lexsort, non_dominated_sort
from ...ops import random as rnd
from ...utils.common import cos_dist
from .common import MOAlgorithm


def theta_nd_sort(obj, w, mask):
    n, nw = obj.shape[0], w.shape[0]
    norm = torch.linalg.norm(obj, dim=1, keepdim=True)
    cosine = cos_dist(obj, w).clamp(-1, 1)
    d1 = norm * cosine
    d2 = norm * torch.sqrt(torch.clamp(1 - cosine**2, min=0))
    cls = torch.argmin(d2, 1)
    theta = torch.where((w > 1e-4).sum(1) == 1, torch.full((nw,), 1e6, device=w.device), torch.full((nw,), 5.0, device=w.device))
    val = d1.gather(1, cls[:, None])[:, 0] + theta[cls] * d2.gather(1, cls[:, None])[:, 0]
    big = nw + 1
    c = torch.where(mask, cls, torch.full_like(cls, big))
    o = torch.argsort(val, stable=True)
    o = o[torch.argsort(c[o], stable=True)]
    c_o = c[o]
    pos = torch.arange(n, device=obj.device) - torch.searchsorted(c_o, c_o)
    t_rank = torch.empty(n, dtype=torch.float32, device=obj.device)
    t_rank[o] = (pos + 1).to(torch.float32)
    return torch.where(mask, t_rank, torch.full_like(t_rank, float("inf")))


class TDEA(MOAlgorithm):
    # decision-axis state sharding (P2): variation per global column, θ-dominance selection
    # from the replicated objectives
    column_separable = True

    def __init__(self, lb, ub, n_objs, pop_size, mutation_op=None, crossover_op=None):
        super().__init__(lb, ub, n_objs, pop_size, mutation_op, crossover_op)
        self.sample = UniformSampling(pop_size, n_objs)

    def setup(self, key):
        key, k1, k2 = rnd.split(key, 3)
        w, _ = self.sample(k2)
        w = w.to(self.lb.device)
        self.pop_size = w.shape[0]
        pop = self._init_pop(k1)
        z = torch.zeros(self.n_objs, device=pop.device)
        return State(population=pop, fitness=torch.zeros((self.pop_size, self.n_objs), device=pop.device), next_generation=pop,
                     w=w, z=z, z_nad=z.clone(), key=key)

    def init_tell(self, state, fitness):
        return state.update(fitness=fitness, z=fitness.min(0).values, z_nad=fitness.max(0).values)

    def ask(self, state):
        key, sel_key, x_key, mut_key = rnd.split(state.key, 4)
        pool = rnd.randint(sel_key, (self.pop_size,), 0, self.pop_size).to(state.population.device)
        off = self._variation(x_key, mut_key, state.population[pool], clip=False)
        return off, state.update(next_generation=off, key=key)

    def tell(self, state, fitness):
        N, m = self.pop_size, self.n_objs
        pop = torch.cat([state.population, state.next_generation], 0)
        obj = torch.cat([state.fitness, fitness], 0)
        rank = non_dominated_sort(obj, until=N + 1)
        worst = torch.sort(rank).values[N]
        mask = rank <= worst
        z = torch.minimum(state.z, obj.min(0).values)
        w1 = torch.where(torch.eye(m, dtype=torch.bool, device=obj.device), 1.0, 1e-6)
        asf = (torch.abs((obj[None] - z) / (state.z_nad - z)) / w1[:, None, :]).amax(-1)  # (m, n)
        ext = torch.argmin(asf, 1)
        sol, info = torch.linalg.solve_ex(obj[ext] - z, torch.ones((m, 1), device=obj.device))
        a = z + 1 / sol[:, 0]
        bad = (info != 0) | torch.isnan(a).any() | (a <= z).any()
        z_nad = torch.where(bad, obj.max(0).values, a)
        norm = (obj - z) / (z_nad - z)
        t_rank = theta_nd_sort(norm, state.w, mask)
        idx = lexsort([t_rank, rank.to(t_rank.dtype)])[:N]
        return state.update(population=pop[idx], fitness=obj[idx], z=z, z_nad=z_nad)
