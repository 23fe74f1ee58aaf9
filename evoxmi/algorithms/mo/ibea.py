"""IBEA (Zitzler & Künzli 2004; reference ``algorithms/mo/ibea.py:21-132``).

I_ε+ indicator fitness and iterative removal of the worst individual with fitness
correction.  The removal loop has a fixed trip count (N) and no host
synchronisation, so it stays on the device (and inside a hipGraph).
"""
from __future__ import annotations

import torch

from ...core import State
from ...operators import selection
from ...ops import random as rnd
from ...utils.common import cal_max
from .common import MOAlgorithm


def cal_fitness(pop_obj, kappa):
    # the reference normalises by the scalar min/max over *all* objectives (ibea.py:23-26)
    mn, mx = pop_obj.min(), pop_obj.max()
    obj = (pop_obj - mn) / (mx - mn)
    I = cal_max(obj, obj)
    C = torch.abs(I).max(0).values
    fitness = (-torch.exp(-I / C[None, :] / kappa)).sum(0) + 1
    return fitness, I, C


def ibea_truncate(fitness, I, C, kappa, n_remove):
    """Remove ``n_remove`` individuals one by one; returns the survivor mask."""
    f = fitness.clone()
    removed = torch.zeros_like(f, dtype=torch.bool)
    for _ in range(n_remove):
        x = torch.argmin(f)
        row = I.index_select(0, x.reshape(1))[0]
        cx = C.index_select(0, x.reshape(1))[0]
        f = f + torch.exp(-row / cx / kappa)
        f = f.scatter(0, x.reshape(1), f.max().reshape(1))
        removed = removed.scatter(0, x.reshape(1), torch.ones(1, dtype=torch.bool, device=f.device))
    return ~removed


class IBEA(MOAlgorithm):
    column_separable = True  # variation per global column, selection by the replicated fitness

    def __init__(self, lb, ub, n_objs, pop_size, kappa=0.05, mutation_op=None, crossover_op=None):
        super().__init__(lb, ub, n_objs, pop_size, mutation_op, crossover_op)
        self.kappa = kappa
        self.selection = selection.Tournament(n_round=pop_size)

    def ask(self, state):
        key, sel_key, x_key, mut_key = rnd.split(state.key, 4)
        fit = cal_fitness(state.fitness, self.kappa)[0]
        selected, _ = self.selection(sel_key, state.population, -fit)
        off = self._variation(x_key, mut_key, selected, clip=False)
        return off, state.update(next_generation=off, key=key)

    def tell(self, state, fitness):
        merged_pop = torch.cat([state.population, state.next_generation], 0)
        merged_obj = torch.cat([state.fitness, fitness], 0)
        f, I, C = cal_fitness(merged_obj, self.kappa)
        keep = ibea_truncate(f, I, C, self.kappa, merged_obj.shape[0] - self.pop_size)
        idx = torch.argsort((~keep).to(torch.int64), stable=True)[: self.pop_size]
        return state.update(population=merged_pop[idx], fitness=merged_obj[idx])
