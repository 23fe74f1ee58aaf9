"""BiGE — bi-goal evolution (Li et al. 2015; reference ``algorithms/mo/bige.py:64-142``).

Each solution is mapped to (proximity = Σ normalised objectives, crowding = sharing
over a niche radius r = 1/N^{1/m}); mating and the last-front truncation use
non-dominated sorting in that bi-goal space.  The reference's ``ask`` estimates the
bi-goal values from the *decision vectors* (``bige.py:110``); the objectives are used
here, as in the method.
"""
from __future__ import annotations

import torch

from ...operators import selection
from ...operators.selection.non_dominate import non_dominated_sort
from ...ops import random as rnd
from .common import MOAlgorithm


def estimate(fit, mask):
    n = mask.sum().to(torch.float32)
    m = fit.shape[1]
    r = 1 / n ** (1 / m)
    big = torch.full_like(fit, float("inf"))
    f_max = torch.where(mask[:, None], fit, -big).max(0).values
    f_min = torch.where(mask[:, None], fit, big).min(0).values
    normed = (fit - f_min) / (f_max - f_min).clamp(min=1e-6)
    normed = torch.where(mask[:, None], normed, torch.full_like(normed, float(m)))
    pr = normed.sum(1)
    dis = torch.cdist(normed, normed)
    ge = (pr[:, None] >= pr[None, :]).to(fit.dtype)
    gt = (pr[:, None] > pr[None, :]).to(fit.dtype)
    sh = ((dis < r).to(fit.dtype) * 0.5 * ((1 + ge + gt) * (1 - dis / r))) ** 2
    cd = torch.sqrt(torch.clamp(sh.sum(1) - sh.diagonal(), min=0))
    bi = torch.stack([pr, cd], 1)
    return torch.where(mask[:, None], bi, torch.full_like(bi, float("inf")))


class BiGE(MOAlgorithm):
    def __init__(self, lb, ub, n_objs, pop_size, mutation_op=None, crossover_op=None):
        super().__init__(lb, ub, n_objs, pop_size, mutation_op, crossover_op)
        self.selection = selection.Tournament(pop_size)

    def ask(self, state):
        k0, k1, k2, k3 = rnd.split(state.key, 4)
        bi = estimate(state.fitness, torch.ones(self.pop_size, dtype=torch.bool, device=state.fitness.device))
        selected, _ = self.selection(k1, state.population, non_dominated_sort(bi).to(torch.float32))
        off = self._variation(k2, k3, selected)
        return off, state.update(next_generation=off, key=k0)

    def tell(self, state, fitness):
        merged_pop = torch.cat([state.population, state.next_generation], 0)
        merged_fit = torch.cat([state.fitness, fitness], 0)
        rank = non_dominated_sort(merged_fit)
        order = torch.argsort(rank, stable=True)
        rank, pop, fit = rank[order], merged_pop[order], merged_fit[order]
        last = rank[self.pop_size]
        bi_rank = non_dominated_sort(estimate(fit, rank == last))
        fin = torch.where(rank >= last, bi_rank, torch.full_like(bi_rank, -1))
        idx = torch.argsort(fin, stable=True)[: self.pop_size]
        return state.update(population=pop[idx], fitness=fit[idx])
