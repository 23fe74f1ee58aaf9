"""NSGA-III (Deb & Jain 2014; reference ``algorithms/mo/nsga3.py:27-211``).

Normalisation by the ideal point and the hyperplane through the extreme points
(falling back to the worst point when the extremes are degenerate), association with
Das–Dennis reference points by perpendicular distance, and niche-preserving
selection from the last front.

The reference fills the remaining K slots with a sequential ``while_loop`` (pick the
niche with the smallest count, lowest index first; take its closest candidate when
the niche was empty, a random one otherwise; increment).  That greedy order is
exactly the lexicographic order of the pairs (ρ_j + k, j) over niches j and their
k-th last-front member, so the loop is replaced by one sort: each candidate gets its
within-niche position k (closest first for empty niches, random otherwise) and the K
smallest (ρ_j + k, j) are kept.  Same distribution, no data-dependent loop.
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


class NSGA3(MOAlgorithm):
    column_separable = True  # variation per global column, selection by the replicated fitness

    def __init__(self, lb, ub, n_objs, pop_size, selection_op=None, mutation_op=None, crossover_op=None):
        super().__init__(lb, ub, n_objs, pop_size, mutation_op, crossover_op)
        self.selection = selection_op if selection_op is not None else selection.UniformRand(1)
        self.ref = UniformSampling(pop_size, n_objs)()[0].to(lb.device)

    def ask(self, state):
        key, mut_key, x_key = rnd.split(state.key, 3)
        off = self._variation(x_key, mut_key, state.population)
        return off, state.update(next_generation=off, key=key)

    def tell(self, state, fitness):
        N, m = self.pop_size, self.n_objs
        merged_pop = torch.cat([state.population, state.next_generation], 0)
        merged_fit = torch.cat([state.fitness, fitness], 0)
        n = merged_fit.shape[0]
        rank = non_dominated_sort(merged_fit, until=N + 1)
        last_rank = torch.sort(rank).values[N]  # 0-d view: no host sync (capturable)
        valid = rank <= last_rank
        inf = torch.full_like(merged_fit, float("inf"))
        ideal = torch.where(valid[:, None], merged_fit, inf).min(0).values
        Fn = merged_fit - ideal
        weight = torch.eye(m, device=Fn.device) + 1e-6
        asf = (Fn[None, :, :] / weight[:, None, :]).amax(-1)  # (m, n)
        asf = torch.where(valid[None, :], asf, torch.full_like(asf, float("inf")))
        extreme = Fn[torch.argmin(asf, 1)]
        sol, info = torch.linalg.solve_ex(extreme, torch.ones(m, 1, device=Fn.device))
        intercept = 1.0 / sol[:, 0]
        worst = torch.where(valid[:, None], Fn, -inf).max(0).values
        ok = (info == 0) & torch.isfinite(intercept).all() & (intercept > 1e-6).all()
        nadir = torch.where(ok, intercept, worst)
        Fn = Fn / nadir
        cosine = cos_dist(Fn, self.ref).clamp(-1, 1)
        dist = torch.linalg.norm(Fn, dim=-1, keepdim=True) * torch.sqrt(torch.clamp(1 - cosine**2, min=0))
        group_dist, group = dist.min(1)
        R = self.ref.shape[0]
        front = rank < last_rank
        last = rank == last_rank
        rho = torch.bincount(group[front], minlength=R)
        K = N - int(front.sum())
        cand = torch.nonzero(last).flatten()
        g = group[cand]
        u = rnd.uniform(state.key, (cand.shape[0],)).to(Fn.device)
        # the closest member of an empty niche goes first
        gd = group_dist[cand]
        big = torch.full((R,), float("inf"), device=Fn.device).scatter_reduce(0, g, gd, "amin")
        first = (rho[g] == 0) & (gd == big[g])
        key_in = torch.where(first, torch.full_like(u, -1.0), u)
        o = lexsort_pair(g, key_in)  # candidates ordered by (niche, key)
        g_o = g[o]
        starts = torch.searchsorted(g_o, g_o, right=False)
        k = torch.arange(g_o.shape[0], device=Fn.device) - starts
        level = rho[g_o] + k
        pick = lexsort_pair(level, g_o.to(torch.float32))[:K]
        chosen = cand[o[pick]]
        keep = front.clone()
        keep[chosen] = True
        idx = torch.nonzero(keep).flatten()[:N]
        key, _ = rnd.split(state.key)
        return state.update(population=merged_pop[idx], fitness=merged_fit[idx], key=key)


def lexsort_pair(primary, secondary):
    """Order by (primary, secondary) ascending, stable."""
    o = torch.argsort(secondary, stable=True)
    return o[torch.argsort(primary[o], stable=True)]
