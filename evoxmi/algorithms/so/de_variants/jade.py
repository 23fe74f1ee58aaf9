"""JaDE — adaptive DE with optional external archive (reference ``de_variants/jade.py:19-204``).

current-to-pbest/1/bin with F ~ Cauchy(F_u, 0.1), CR ~ N(CR_u, 0.1) clipped to
[0, 1]; after each generation F_u ← (1−c)F_u + c·Lehmer(S_F) and
CR_u ← (1−c)CR_u + c·mean(S_CR) over the successful parameters; replaced parents go
to the archive slot of their index.
"""
from __future__ import annotations

import torch

from ....parallel.dim_sharded import ColumnSeparable
from ....core import Algorithm
from ....ops import random as rnd
from . import common as C


class JaDE(ColumnSeparable, Algorithm):
    # decision-axis state sharding (P2): current-to-pbest/1 + archive trials drawn per global
    # column (generate_trials cols=), F/CR and the archive's row choice replicated
    column_separable = True
    dim_fields = ("population", "trial_vectors", "archive")

    def __init__(self, lb, ub, pop_size=100, diff_padding_num=3, differential_weight=None, cross_probability=None, c=0.1,
                 p=0.05, with_archive=1):
        super().__init__()
        self.dim = lb.shape[0]
        self.lb, self.ub = lb, ub
        self.pop_size = pop_size
        self.batch_size = pop_size
        self.diff_padding_num = diff_padding_num
        self.c = c
        self.p = p
        self.with_archive = with_archive

    def setup(self, key):
        state_key, init_key = rnd.split(key)
        pop = C.init_population(init_key, self.pop_size, self.lb, self.ub)
        dev = pop.device
        N = self.pop_size
        return C.base_state(state_key, pop, trial_vectors=torch.zeros_like(pop), F_u=C.scalar(0.5, dev), CR_u=C.scalar(0.5, dev),
                            F_vect=torch.zeros(N, device=dev), CR_vect=torch.zeros(N, device=dev), archive=pop.clone())

    def ask(self, state):
        key, k_trial, k_f, k_cr = rnd.split(state.key, 4)
        dev = state.population.device
        N = self.pop_size
        F = torch.clamp(rnd.cauchy(k_f, (N,)).to(dev) * 0.1 + state.F_u, 0, 1)
        CR = torch.clamp(rnd.normal(k_cr, (N,)).to(dev) * 0.1 + state.CR_u, 0, 1)
        cur = torch.arange(N, device=dev)
        c0, own, d = self.cols()
        trials, _ = C.generate_trials(k_trial, state.population, state.fitness, state.best_index, cur, C.current2pbest_1_bin, F,
                                      CR, self.diff_padding_num, self.col_vec(self.lb), self.col_vec(self.ub), p=self.p,
                                      archive=state.archive if self.with_archive else None, cols=(c0, d))
        return trials, state.update(trial_vectors=trials, key=key, F_vect=F, CR_vect=CR)

    def tell(self, state, trial_fitness):
        pop, fit, ok = C.greedy_replace(state.population, state.fitness, state.trial_vectors, trial_fitness, strict=True)
        any_ok = ok.any()
        F_l = C.lehmer_update(ok, state.F_vect)
        CR_m = torch.nanmean(torch.where(ok, state.CR_vect, torch.full_like(state.CR_vect, float("nan"))))
        F_u = torch.where(any_ok, (1 - self.c) * state.F_u + self.c * F_l, state.F_u)
        CR_u = torch.where(any_ok, (1 - self.c) * state.CR_u + self.c * CR_m, state.CR_u)
        archive = torch.where(ok[:, None], state.population, state.archive)
        return state.update(population=pop, fitness=fit, best_index=torch.argmin(fit), F_u=F_u, CR_u=CR_u, archive=archive)
