"""HypE — hypervolume estimation algorithm (Bader & Zitzler 2011; reference ``algorithms/mo/hype.py:21-147``).

Monte-Carlo estimate of each point's shared hypervolume contribution
(``α_i = Π_{j<i}(k−j)/(n−j) / i`` weighting of samples dominated by i points),
binary tournament on it, and (rank, −contribution) truncation of the worst front.
The reference's ``ask`` never advances the key (``hype.py:122``); here it does.
"""
from __future__ import annotations

import torch

from ...core import State
from ...operators import selection
from ...operators.selection.non_dominate import lexsort, non_dominated_sort
from ...ops import geom
from ...ops import random as rnd
from .common import MOAlgorithm


def cal_hv(points, ref, k, n_sample, key):
    n, m = points.shape
    j = torch.arange(1, n, dtype=torch.float32, device=points.device)
    alpha = torch.cumprod(torch.cat([torch.ones(1, device=points.device), (k - j) / (n - j)]), 0) / torch.arange(1, n + 1, device=points.device)
    f_min = points.min(0).values
    samples = rnd.uniform(key, (n_sample, m)).to(points.device) * (ref - f_min) + f_min
    # K18: per-sample dominator counts, then per-point Σ α[count − 1] (two kernels on the GPU)
    cnt = geom.hv_count(samples, points, strict=False)
    f = geom.hv_contrib(samples, points, cnt, alpha)
    return f * torch.prod(ref - f_min) / n_sample


class HypE(MOAlgorithm):
    column_separable = True  # variation per global column, selection by the replicated fitness

    def __init__(self, lb, ub, n_objs, pop_size, n_sample=10000, mutation_op=None, crossover_op=None):
        super().__init__(lb, ub, n_objs, pop_size, mutation_op, crossover_op)
        self.n_sample = n_sample
        self.selection = selection.Tournament(n_round=pop_size, multi_objective=True)

    def setup(self, key):
        return super().setup(key).update(ref_point=torch.zeros(self.n_objs, device=self.lb.device))

    def init_tell(self, state, fitness):
        return state.update(fitness=fitness, ref_point=torch.zeros(self.n_objs, device=fitness.device) + fitness.max() * 1.2)

    def ask(self, state):
        key, sub, sel_key, x_key, mut_key = rnd.split(state.key, 5)
        hv = cal_hv(state.fitness, state.ref_point, self.pop_size, self.n_sample, sub)
        selected, _ = self.selection(sel_key, state.population, -hv[:, None])
        off = self._variation(x_key, mut_key, selected, clip=False)
        return off, state.update(next_generation=off, key=key)

    def tell(self, state, fitness):
        merged_pop = torch.cat([state.population, state.next_generation], 0)
        merged_obj = torch.cat([state.fitness, fitness], 0)
        n = merged_obj.shape[0]
        rank = non_dominated_sort(merged_obj)
        worst = rank.max()
        key, sub = rnd.split(state.key)
        hv = cal_hv(merged_obj, state.ref_point, n, self.n_sample, sub)
        dis = torch.where(rank == worst, hv, torch.full_like(hv, -float("inf")))
        idx = lexsort([-dis, rank.to(dis.dtype)])[: self.pop_size]
        return state.update(population=merged_pop[idx], fitness=merged_obj[idx], key=key)
