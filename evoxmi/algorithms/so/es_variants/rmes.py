"""RM-ES — rank-m ES with a P-matrix memory (Li & Zhang 2017; reference ``es_variants/rmes.py:22-202``).

CMA-ES with a sparse-plus-low-rank C update, an evolution-path memory P with
generation gaps and the rank-success rule.  Deviation: the reference's
``_update_mean`` re-sorts the population by its *first coordinate* and, with the
default ``mean_decay = 0``, keeps the mean fixed forever (``rmes.py:109-114``); here
the mean is the fitness-weighted elite recombination, blended with the old mean by
``mean_decay``.
"""
from __future__ import annotations

import torch

from ._cma_base import TextbookCMA
from ._common import sort_by_key


class RMES(TextbookCMA):
    def __init__(self, center_init, init_stdev, pop_size=None, recombination_weights=None, cm=1, elite_ratio=0.5,
                 memory_size=10, mean_decay=0, sparse_threshold=0.01, t_uncorr=10):
        super().__init__(center_init, init_stdev, pop_size, recombination_weights, cm)
        self.elite_ratio = elite_ratio
        self.elite_popsize = max(1, int(self.pop_size * self.elite_ratio))
        self.memory_size = memory_size
        self.mean_decay = mean_decay
        self.sparse_threshold = sparse_threshold
        self.c_sigma = (self.mueff + 2) / (self.dim + self.mueff + 5)
        self.t_uncorr = t_uncorr
        self.q_star, self.c_s, self.d_sigma, self.s_rank_rate = 0.5, 0.3, 1.0, 0.0

    def setup(self, key):
        st = super().setup(key)
        dev = st.mean.device
        return st.update(P=torch.zeros((self.dim, self.memory_size), device=dev), t_gap=torch.zeros(self.memory_size, device=dev),
                         s_rank_rate=torch.zeros((), device=dev), fitness_archive=torch.full((self.pop_size,), 1e20, device=dev),
                         p_sigma=torch.zeros(self.dim, device=dev))

    def _update_mean(self, mean, population):
        weighted = self.weights @ population[: self.mu]
        return (1 - self.mean_decay) * weighted + self.mean_decay * mean

    def _sparse_plus_low_rank_update(self, y, pc):
        o = torch.outer(y.mean(0), pc)
        return torch.where(o.abs() > self.sparse_threshold, o, torch.zeros_like(o)) + torch.outer(pc, pc)

    def _update_C(self, C, pc, sigma, population, old_mean, hsig):
        y = (population[: self.mu] - old_mean) / sigma
        return ((1 - self.c1 - self.cmu) * C + self.c1 * (self._sparse_plus_low_rank_update(y, pc) + (1 - hsig) * self.cc * (2 - self.cc) * C)
                + self.cmu * (y.T * self.weights) @ y)

    def _update_P_matrix(self, P, p_sigma, t_gap, gen):
        m = P.shape[1]
        T_min = (t_gap[1:] - t_gap[:-1]).min()
        push = (T_min > self.t_uncorr) | (gen < m)
        P_c1 = torch.cat([P[:, 1:], P[:, -1:]], 1)
        t_c1 = torch.cat([t_gap[1:], t_gap[-1:]])
        i_min = torch.argmin(t_gap[:-1] - t_gap[1:])
        j = torch.arange(m, device=P.device)
        shift = (j >= i_min) & (j < m - 1)
        src = torch.where(shift, j + 1, j)
        P_c2, t_c2 = P[:, src], t_gap[src]
        P1 = torch.where(push, P_c1, P_c2)
        t1 = torch.where(push, t_c1, t_c2)
        P_new = torch.cat([P1[:, :-1], p_sigma[:, None]], 1)
        t_new = torch.cat([t1[:-1], gen.to(t1.dtype).reshape(1)])
        return P_new, t_new

    def _rank_success_rule(self, fitness, fitness_archive):
        k = self.weights.shape[0]
        n = fitness.shape[0]
        allf = torch.cat([fitness, fitness_archive])
        ranks = torch.empty(2 * n, device=fitness.device)
        ranks[torch.argsort(allf, stable=True)] = torch.arange(2 * n, dtype=torch.float32, device=fitness.device)
        rc = torch.sort(ranks[:n]).values[:k]
        rl = torch.sort(ranks[n:]).values[:k]
        q = (self.weights * (rl - rc)).sum() / k
        return (1 - self.c_s) * self.s_rank_rate + self.c_s * (q - self.q_star)

    def tell(self, state, fitness):
        sfit, population = sort_by_key(fitness, state.population)
        new_state = super().tell(state, fitness)
        mean = new_state.mean
        p_sigma = (1 - self.c_sigma) * state.p_sigma + (self.c_sigma * (2 - self.c_sigma) * self.mueff) ** 0.5 * (mean - state.mean) / state.sigma
        P, t_gap = self._update_P_matrix(state.P, state.p_sigma, state.t_gap, state.count_iter)
        return new_state.update(p_sigma=p_sigma, P=P, t_gap=t_gap, s_rank_rate=self._rank_success_rule(sfit, state.fitness_archive),
                                fitness_archive=sfit)
