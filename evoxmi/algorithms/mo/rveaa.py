"""RVEA* (RVEA with reference-vector regeneration; reference ``algorithms/mo/rveaa.py:63-215``).

A second set of reference vectors is regenerated at random wherever no
non-dominated solution is associated; the population has 2N NaN-padded slots; on
the penultimate generation the survivors are batch-truncated to N by removing the
most crowded (largest maximum cosine to another solution).
"""
from __future__ import annotations

import torch

from ...core import State
from ...operators import selection
from ...operators.sampling import UniformSampling
from ...operators.selection.non_dominate import non_dominated_sort
from ...ops import random as rnd
from ...utils.common import cos_dist
from .common import MOAlgorithm


def rv_regeneration(pop_obj, v, key):
    obj = pop_obj - torch.nan_to_num(pop_obj, nan=float("inf")).min(0).values
    cosine = torch.nan_to_num(cos_dist(obj, v), nan=-float("inf"))
    assoc = torch.argmax(cosine, 1)
    valid_row = ~torch.isnan(pop_obj).any(1)
    hit = torch.zeros(v.shape[0], device=v.device).scatter_add_(0, assoc, valid_row.to(torch.float32))
    rand = rnd.uniform(key, tuple(v.shape)).to(v.device) * torch.nan_to_num(obj, nan=-float("inf")).max(0).values
    return torch.where((hit == 0)[:, None], rand, v)


def batch_truncation(pop, obj):
    n = pop.shape[0] // 2
    cosine = cos_dist(obj, obj)
    cosine = cosine.masked_fill(torch.eye(cosine.shape[0], dtype=torch.bool, device=obj.device), 0)
    top = torch.nan_to_num(cosine, nan=-float("inf")).max(1).values  # most similar neighbour
    worst = torch.argsort(-top, stable=True)[:n]  # most crowded first (NaN rows last)
    keep = torch.ones(pop.shape[0], dtype=torch.bool, device=pop.device)
    keep[worst] = False
    nan = torch.full_like(pop, float("nan"))
    return torch.where(keep[:, None], pop, nan), torch.where(keep[:, None], obj, torch.full_like(obj, float("nan")))


class RVEAa(MOAlgorithm):
    def __init__(self, lb, ub, n_objs, pop_size, alpha=2, fr=0.1, max_gen=100, selection_op=None, mutation_op=None, crossover_op=None):
        super().__init__(lb, ub, n_objs, pop_size, mutation_op, crossover_op)
        self.alpha, self.fr, self.max_gen = alpha, fr, max_gen
        self.selection = selection_op if selection_op is not None else selection.ReferenceVectorGuided()
        self.sampling = UniformSampling(pop_size, n_objs)

    def setup(self, key):
        key, k1, k2, k3 = rnd.split(key, 4)
        v0 = self.sampling(k1)[0].to(self.lb.device)
        self.pop_size = v0.shape[0]
        pop0 = self._init_pop(k2)
        dev = pop0.device
        pop = torch.cat([pop0, torch.full_like(pop0, float("nan"))])
        v = torch.cat([v0, rnd.uniform(k3, (self.pop_size, self.n_objs)).to(dev)])
        return State(population=pop, fitness=torch.zeros((2 * self.pop_size, self.n_objs), device=dev), next_generation=pop0,
                     reference_vector=v, init_v=v0, key=key, gen=torch.zeros((), dtype=torch.int64, device=dev))

    def init_ask(self, state):
        return state.population, state

    def ask(self, state):
        key, sub, x_key, mut_key = rnd.split(state.key, 4)
        valid = ~torch.isnan(state.population).all(1)
        order = torch.argsort((~valid).to(torch.int64), stable=True)
        r = torch.floor(rnd.uniform(sub, (self.pop_size,)).to(valid.device) * valid.sum().clamp(min=1)).long()
        off = self._variation(x_key, mut_key, state.population[order[r]])
        return off, state.update(next_generation=off, key=key)

    def tell(self, state, fitness):
        key, sub = rnd.split(state.key)
        gen = state.gen + 1
        N = self.pop_size
        v = state.reference_vector
        pop = torch.cat([state.population, state.next_generation])
        obj = torch.cat([state.fitness, fitness])
        rank = non_dominated_sort(torch.nan_to_num(obj, nan=float("inf")))
        nd = (rank == 0) & ~torch.isnan(obj).any(1)
        obj = torch.where(nd[:, None], obj, torch.full_like(obj, float("nan")))
        pop = torch.where(nd[:, None], pop, torch.full_like(pop, float("nan")))
        surv, surv_fit = self.selection(pop, obj, v, (gen.to(torch.float32) / self.max_gen) ** self.alpha)
        period = int(round(1 / self.fr))
        span = torch.nan_to_num(surv_fit, nan=-float("inf")).max(0).values - torch.nan_to_num(surv_fit, nan=float("inf")).min(0).values
        v_adapt = torch.where((gen % period) == 0, state.init_v * span, v[:N])
        v = torch.cat([v_adapt, rv_regeneration(surv_fit, v[N:], sub)])
        if int(gen) + 1 == self.max_gen:
            surv, surv_fit = batch_truncation(surv, surv_fit)
        return state.update(population=surv, fitness=surv_fit, reference_vector=v, gen=gen, key=key)
