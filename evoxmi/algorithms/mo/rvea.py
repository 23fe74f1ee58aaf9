"""RVEA (Cheng et al. 2016; reference ``algorithms/mo/rvea.py:17-140``).

Angle-penalised distance selection per reference vector (NaN-padded population of
static size), reference-vector adaptation to the objective ranges every 1/fr
generations.  Mating picks uniformly among the non-padding rows.
"""
from __future__ import annotations

import torch

from ...core import State
from ...operators import selection
from ...operators.sampling import UniformSampling
from ...ops import random as rnd
from .common import MOAlgorithm


class RVEA(MOAlgorithm):
    # decision-axis state sharding (P2): SBX + PM per global column (ColumnVariation), the
    # APD selection and the reference-vector adaptation use the replicated objectives only
    column_separable = True

    def __init__(self, lb, ub, n_objs, pop_size, alpha=2, fr=0.1, max_gen=100, selection_op=None, mutation_op=None, crossover_op=None):
        super().__init__(lb, ub, n_objs, pop_size, mutation_op, crossover_op)
        self.alpha, self.fr, self.max_gen = alpha, fr, max_gen
        self.selection = selection_op if selection_op is not None else selection.ReferenceVectorGuided()
        self.sampling = UniformSampling(pop_size, n_objs)

    def setup(self, key):
        key, k1, k2 = rnd.split(key, 3)
        v = self.sampling(k2)[0].to(self.lb.device)
        self.pop_size = v.shape[0]
        pop = self._init_pop(k1)
        return State(population=pop, fitness=torch.zeros((self.pop_size, self.n_objs), device=pop.device), next_generation=pop,
                     reference_vector=v, init_v=v.clone(), key=key, gen=torch.zeros((), dtype=torch.int64, device=pop.device))

    def ask(self, state):
        key, sub, x_key, mut_key = rnd.split(state.key, 4)
        valid = ~torch.isnan(state.population).all(1)
        order = torch.argsort((~valid).to(torch.int64), stable=True)  # valid rows first
        n_valid = valid.sum().clamp(min=1)
        r = torch.floor(rnd.uniform(sub, (self.pop_size,)).to(valid.device) * n_valid).long()
        parents = state.population[order[r]]
        off = self._variation(x_key, mut_key, parents)
        return off, state.update(next_generation=off, key=key)

    def tell(self, state, fitness):
        gen = state.gen + 1
        merged_pop = torch.cat([state.population, state.next_generation], 0)
        merged_fit = torch.cat([state.fitness, fitness], 0)
        theta = (gen.to(torch.float32) / self.max_gen) ** self.alpha
        surv, surv_fit = self.selection(merged_pop, merged_fit, state.reference_vector, theta)
        period = int(round(1 / self.fr))
        span = torch.nan_to_num(surv_fit, nan=-float("inf")).max(0).values - torch.nan_to_num(surv_fit, nan=float("inf")).min(0).values
        v = torch.where((gen % period) == 0, state.init_v * span, state.reference_vector)
        return state.update(population=surv, fitness=surv_fit, reference_vector=v, gen=gen)
