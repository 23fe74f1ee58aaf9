"""SRA — stochastic ranking algorithm (Li et al. 2016; reference ``algorithms/mo/sra.py:115-191``).

Two indicators — I_ε+ fitness (I1) and shift-based density (I2) — are balanced by
stochastic ranking (a bubble sort choosing the comparison indicator at random with
probability pc ∈ [0.4, 0.6]).  The bubble sort is sequential by nature; it runs as a
small host-side C++ op (``evoxmi::stochastic_ranking``).  The reference fills the SDE
distance matrix only below the diagonal (``sra.py:96-106``), so its I2 ignores later
individuals; here I2 is the SDE nearest-neighbour distance over all j ≠ i.
"""
from __future__ import annotations

import math

import torch

from ...operators import crossover
from ...ops import _ext
from ...ops import random as rnd
from ...utils.common import cal_max
from .common import MOAlgorithm


def stochastic_ranking(I1, I2, u, pc):
    if _ext.available():
        return _ext.ops().stochastic_ranking(I1, I2, u, float(pc)).to(I1.device)
    n = I1.shape[0]
    a, b, uu = I1.tolist(), I2.tolist(), u.tolist()
    r = list(range(n))
    for _ in range((n + 1) // 2):
        swapped = False
        for j in range(n - 1):
            k = a if uu[j] < pc else b
            if k[r[j]] < k[r[j + 1]]:
                r[j], r[j + 1] = r[j + 1], r[j]
                swapped = True
        if not swapped:
            break
    return torch.tensor(r, device=I1.device)


def sde_distance(obj):
    n = obj.shape[0]
    d = torch.sqrt((torch.clamp(obj[None, :, :] - obj[:, None, :], min=0) ** 2).sum(-1))  # d[i, j] = ‖max(o_j − o_i, 0)‖
    return d.masked_fill(torch.eye(n, dtype=torch.bool, device=obj.device), float("inf")).min(1).values


class SRA(MOAlgorithm):
    def __init__(self, lb, ub, n_objs, pop_size, mutation_op=None, crossover_op=None):
        super().__init__(lb, ub, n_objs, pop_size, mutation_op, crossover_op if crossover_op is not None else crossover.SimulatedBinary(type=2))

    def ask(self, state):
        key, sel_key, x_key, mut_key = rnd.split(state.key, 4)
        pool = rnd.randint(sel_key, (self.pop_size * 2,), 0, self.pop_size).to(state.population.device)
        off = self.mutation(mut_key, self.crossover(x_key, state.population[pool]))
        return off, state.update(next_generation=off, key=key)

    def tell(self, state, fitness):
        merged_pop = torch.cat([state.population, state.next_generation], 0)
        merged_fit = torch.cat([state.fitness, fitness], 0)
        key, k_pc, k_env = rnd.split(state.key, 3)
        pc = float(rnd.uniform(k_pc, ())) * 0.2 + 0.4
        I = cal_max(merged_fit, merged_fit)
        I1 = (-torch.exp(-I / 0.05)).sum(0) + 1
        I2 = sde_distance(merged_fit)
        u = rnd.uniform(k_env, (merged_fit.shape[0] - 1,))
        idx = stochastic_ranking(I1, I2, u, pc)[: self.pop_size]
        return state.update(population=merged_pop[idx], fitness=merged_fit[idx], key=key)
