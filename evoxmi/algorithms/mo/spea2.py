"""SPEA2 (Zitzler et al. 2001; reference ``algorithms/mo/spea2.py:71-158``).

Strength + raw fitness + k-th nearest-neighbour density; environmental selection
keeps the non-dominated set, filled by fitness or truncated by iteratively removing
the individual closest to its nearest neighbour.
"""
from __future__ import annotations

import math

import torch

from ...core import State
from ...operators import selection
from ...ops import random as rnd
from ...utils.common import dominate_relation
from .common import MOAlgorithm


def cal_fitness(obj):
    n = obj.shape[0]
    dom = dominate_relation(obj, obj)  # dom[i, j]: i dominates j
    S = dom.sum(1).to(torch.float32)
    R = (dom.to(torch.float32) * S[:, None]).sum(0)
    dis = torch.cdist(obj, obj)
    dis = dis.masked_fill(torch.eye(n, dtype=torch.bool, device=obj.device), float("inf"))
    k = int(math.floor(math.sqrt(6))) - 1
    D = 1 / (torch.sort(dis, dim=1).values[:, k] + 2)
    return D + R


def truncation(obj, k, mask):
    """Remove ``k`` of the masked points, each time the one whose nearest neighbour is closest."""
    n = obj.shape[0]
    dis = torch.cdist(obj, obj)
    dis = dis.masked_fill(torch.eye(n, dtype=torch.bool, device=obj.device), float("inf"))
    dis = torch.where(mask[:, None] & mask[None, :], dis, torch.full_like(dis, float("inf")))
    keep = torch.ones(n, dtype=torch.bool, device=obj.device)
    for _ in range(k):
        idx = torch.argmin(dis.min(1).values)
        keep[idx] = False
        dis[idx, :] = float("inf")
        dis[:, idx] = float("inf")
    return keep & mask


def truncation_predicated(obj, k, mask, max_k: int):
    """``truncation`` with a device-resident removal count ``k`` (≤ ``max_k``)."""
    n = obj.shape[0]
    inf = float("inf")
    dis = torch.cdist(obj, obj)
    dis = dis.masked_fill(torch.eye(n, dtype=torch.bool, device=obj.device), inf)
    dis = torch.where(mask[:, None] & mask[None, :], dis, torch.full_like(dis, inf))
    keep = torch.ones(n, dtype=torch.bool, device=obj.device)
    col = torch.arange(n, device=obj.device)
    for step in range(max_k):
        act = k > step
        idx = torch.argmin(dis.min(1).values)
        hit = (col == idx) & act
        keep = keep & ~hit
        dis = dis.masked_fill(hit[:, None] | hit[None, :], inf)
    return keep & mask


class SPEA2(MOAlgorithm):
    # decision-axis state sharding (P2): variation per global column, tournament and
    # truncation from the replicated objectives
    column_separable = True

    def __init__(self, lb, ub, n_objs, pop_size, mutation_op=None, crossover_op=None):
        super().__init__(lb, ub, n_objs, pop_size, mutation_op, crossover_op)
        self.selection = selection.Tournament(n_round=pop_size)

    def ask(self, state):
        key, sel_key, x_key, mut_key = rnd.split(state.key, 4)
        selected, _ = self.selection(sel_key, state.population, cal_fitness(state.fitness))
        off = self._variation(x_key, mut_key, selected, clip=False)
        return off, state.update(next_generation=off, key=key)

    def tell(self, state, fitness):
        merged_pop = torch.cat([state.population, state.next_generation], 0)
        merged_fit = torch.cat([state.fitness, fitness], 0)
        sig = cal_fitness(merged_fit)
        mask = sig < 1
        if merged_fit.is_cuda and torch.cuda.is_current_stream_capturing():
            # capturable form: the removal count stays on the device; a fixed N-step loop with
            # predicated updates replaces the data-dependent one, and the branch becomes a select
            num_valid = mask.sum()
            keep = truncation_predicated(merged_fit, num_valid - self.pop_size, mask, self.pop_size)
            key = torch.where(num_valid <= self.pop_size, sig, (~keep).to(sig.dtype))
            order = torch.argsort(key, stable=True)
        else:
            num_valid = int(mask.sum())
            if num_valid <= self.pop_size:
                order = torch.argsort(sig, stable=True)
            else:
                keep = truncation(merged_fit, num_valid - self.pop_size, mask)
                order = torch.argsort((~keep).to(torch.int64), stable=True)
        idx = order[: self.pop_size]
        return state.update(population=merged_pop[idx], fitness=merged_fit[idx])
