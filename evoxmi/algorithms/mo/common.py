"""Shared skeleton of the multi-objective algorithms: random initial population in
the box, ``init_ask``/``init_tell`` evaluation of it, SBX + polynomial-mutation
variation (fused HIP kernels on a GPU), NSGA-II-style environmental selection."""
from __future__ import annotations

import torch

from ...core import Algorithm, State
from ...operators import crossover, mutation
from ...operators.selection.non_dominate import crowding_distance, lexsort, non_dominated_sort
from ...ops import random as rnd


class MOAlgorithm(Algorithm):
    def __init__(self, lb, ub, n_objs, pop_size, mutation_op=None, crossover_op=None):
        super().__init__()
        self.lb, self.ub = lb, ub
        self.n_objs = n_objs
        self.dim = lb.shape[0]
        self.pop_size = pop_size
        self.mutation = mutation_op if mutation_op is not None else mutation.Polynomial((lb, ub))
        self.crossover = crossover_op if crossover_op is not None else crossover.SimulatedBinary()

    def _init_pop(self, key):
        return rnd.uniform(key, (self.pop_size, self.dim)).to(self.lb.device) * (self.ub - self.lb) + self.lb

    def setup(self, key):
        key, sub = rnd.split(key)
        pop = self._init_pop(sub)
        return State(population=pop, fitness=torch.zeros((self.pop_size, self.n_objs), device=pop.device), next_generation=pop, key=key)

    def init_ask(self, state):
        return state.population, state

    def init_tell(self, state, fitness):
        return state.update(fitness=fitness)

    def _variation(self, x_key, mut_key, parents, clip=True):
        off = self.mutation(mut_key, self.crossover(x_key, parents))
        return torch.clamp(off, self.lb, self.ub) if clip else off


def nsga2_select(fitness, n):
    """Indices of the n survivors by (rank, −crowding) (reference ``eagmoead.py:22-30``)."""
    if fitness.is_cuda and fitness.shape[0] <= 8192:
        from ...ops import nds

        return nds.nsga2_survivors(fitness, n, n - 1, until=n)
    rank = non_dominated_sort(fitness, until=n)
    worst = torch.sort(rank).values[n - 1]  # 0-d view: no host sync (capturable)
    cd = crowding_distance(fitness, rank == worst)
    return lexsort([-cd, rank.to(cd.dtype)])[:n]


def weights_and_neighbours(w, T):
    d = torch.cdist(w, w)
    return torch.argsort(d, dim=1, stable=True)[:, :T]
