"""GDE3 (Kukkonen & Lampinen 2005; reference ``algorithms/mo/gde3.py:24-98``):
DE/rand/1/bin offspring (F = 0.49, CR = 0.97) + NSGA-II environmental selection."""
from __future__ import annotations

import torch

from ...operators import crossover
from ...ops import random as rnd
from .common import MOAlgorithm, nsga2_select


class GDE3(MOAlgorithm):
    def __init__(self, lb, ub, n_objs, pop_size, F=0.49, CR=0.97):
        super().__init__(lb, ub, n_objs, pop_size)
        self.F, self.CR = F, CR
        self.de = crossover.DifferentialEvolve(F, CR)

    def ask(self, state):
        k0, k1, k2 = rnd.split(state.key, 3)
        idx = rnd.randint(k1, (3, self.pop_size), 0, self.pop_size).to(state.population.device)
        p = state.population[idx]
        off = torch.clamp(self.de(k2, p[0], p[1], p[2]), self.lb, self.ub)
        return off, state.update(next_generation=off, key=k0)

    def tell(self, state, fitness):
        merged_pop = torch.cat([state.population, state.next_generation], 0)
        merged_fit = torch.cat([state.fitness, fitness], 0)
        idx = nsga2_select(merged_fit, self.pop_size)
        return state.update(population=merged_pop[idx], fitness=merged_fit[idx])
