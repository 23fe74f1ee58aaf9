"""SHADE — success-history adaptive DE (reference ``de_variants/shade.py:18-219``).

Historical memories M_F, M_CR of size H = pop_size; each row samples a memory
slot, F ~ Cauchy(M_F, 0.1), CR ~ N(M_CR, 0.1) clipped; after selection the
improvement-weighted Lehmer mean of successful F and weighted mean of CR are
rolled into slot 0; replaced parents go to the archive; p ~ U(2/N, 0.2).
"""
from __future__ import annotations

import torch

from ....parallel.dim_sharded import ColumnSeparable
from ....core import Algorithm
from ....ops import random as rnd
from . import common as C


class SHADE(ColumnSeparable, Algorithm):
    # decision-axis state sharding (P2): see JaDE
    column_separable = True
    dim_fields = ("population", "trial_vectors", "archive")

    def __init__(self, lb, ub, pop_size=100, diff_padding_num=3, differential_weight=None, cross_probability=None,
                 with_archive=1, p=0.05):
        super().__init__()
        self.dim = lb.shape[0]
        self.lb, self.ub = lb, ub
        self.pop_size = pop_size
        self.batch_size = pop_size
        self.diff_padding_num = diff_padding_num
        self.H = pop_size
        self.p = p
        self.with_archive = with_archive

    def setup(self, key):
        state_key, init_key = rnd.split(key)
        pop = C.init_population(init_key, self.pop_size, self.lb, self.ub)
        dev = pop.device
        N = self.pop_size
        return C.base_state(state_key, pop, trial_vectors=torch.zeros_like(pop),
                            Memory_F=torch.full((self.H,), 0.5, device=dev), Memory_CR=torch.full((self.H,), 0.5, device=dev),
                            F_vect=torch.zeros(N, device=dev), CR_vect=torch.zeros(N, device=dev), archive=pop.clone(),
                            p=C.scalar(self.p, dev))

    def ask(self, state):
        key, k_trial, k_choice, k_f, k_cr = rnd.split(state.key, 5)
        dev = state.population.device
        N = self.pop_size
        ids = rnd.randint(k_choice, (N,), 0, self.H).to(dev)
        F = torch.clamp(rnd.cauchy(k_f, (N,)).to(dev) * 0.1 + state.Memory_F[ids], 0, 1)
        CR = torch.clamp(rnd.normal(k_cr, (N,)).to(dev) * 0.1 + state.Memory_CR[ids], 0, 1)
        cur = torch.arange(N, device=dev)
        c0, own, d = self.cols()
        trials, _ = C.generate_trials(k_trial, state.population, state.fitness, state.best_index, cur, C.current2pbest_1_bin, F,
                                      CR, self.diff_padding_num, self.col_vec(self.lb), self.col_vec(self.ub), p=state.p,
                                      archive=state.archive if self.with_archive else None, cols=(c0, d))
        return trials, state.update(trial_vectors=trials, key=key, F_vect=F, CR_vect=CR)

    def tell(self, state, trial_fitness):
        pop, fit, _ = C.greedy_replace(state.population, state.fitness, state.trial_vectors, trial_fitness, strict=False)
        ok = trial_fitness < state.fitness
        nan = torch.full_like(trial_fitness, float("nan"))
        S_delta = torch.where(ok, state.fitness - trial_fitness, nan)
        w = S_delta / torch.nansum(S_delta)
        M_CR = torch.nansum(w * torch.where(ok, state.CR_vect, nan))
        # no success ⇒ nansum(∅) = 0 is rolled into M_CR (reference shade.py:190-199 behaves so)
        M_F = C.lehmer_update(ok, state.F_vect, w)
        archive = torch.where(ok[:, None], state.population, state.archive)
        p_key, _ = rnd.split(state.key)
        p = rnd.uniform(p_key, (), minval=2 / self.pop_size, maxval=0.2).to(state.population.device)
        return state.update(population=pop, fitness=fit, best_index=torch.argmin(fit), Memory_F=C.roll_in(state.Memory_F, M_F),
                            Memory_CR=C.roll_in(state.Memory_CR, M_CR), archive=archive, p=p)
