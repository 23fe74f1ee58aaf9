"""CoDE — composite trial vector generation (reference ``de_variants/code.py:28-196``).

Every generation each target gets three trials, one per strategy
{rand/1/bin, rand/2/bin, current-to-rand/1 (arith)}, each with an (F, CR) pair
drawn from the pool {(1, .1), (1, .9), (.8, .2)} → 3·B evaluations; the best of
the three competes with the target (``<=``).  All 3·B trials are one fused kernel
launch (per-row strategy codes).
"""
from __future__ import annotations

import torch

from ....core import Algorithm
from ....ops import random as rnd
from . import common as C


class CoDE(Algorithm):
    def __init__(self, lb, ub, pop_size=100, batch_size=None, diff_padding_num=5,
                 param_pool=((1, 0.1), (1, 0.9), (0.8, 0.2)), replace=False):
        super().__init__()
        self.dim = lb.shape[0]
        self.lb, self.ub = lb, ub
        self.pop_size = pop_size
        self.batch_size = batch_size or pop_size
        self.param_pool = torch.as_tensor(param_pool, dtype=torch.float32)
        self.diff_padding_num = diff_padding_num
        self.strategies = torch.tensor([C.rand_1_bin, C.rand_2_bin, C.current2rand_1])
        self.replace = replace

    def setup(self, key):
        state_key, init_key = rnd.split(key)
        pop = C.init_population(init_key, self.pop_size, self.lb, self.ub)
        dev = pop.device
        return C.base_state(state_key, pop, trial_vectors=torch.zeros((3 * self.batch_size, self.dim), device=dev),
                            start_index=C.scalar(0, dev, torch.int64))

    def _cur(self, state):
        return (torch.arange(self.batch_size, device=state.population.device) + state.start_index) % self.pop_size

    def ask(self, state):
        key, k_trial, k_param = rnd.split(state.key, 3)
        dev = state.population.device
        B = self.batch_size
        cur = self._cur(state).repeat(3)
        pids = rnd.randint(k_param, (3 * B,), 0, 3).to(dev)
        params = C.dconst(self.param_pool, dev)[pids]
        strat = C.dconst(self.strategies, dev, torch.int64).repeat_interleave(B, 0)
        trials, _ = C.generate_trials(k_trial, state.population, state.fitness, state.best_index, cur, strat, params[:, 0],
                                      params[:, 1], self.diff_padding_num, self.lb, self.ub)
        return trials, state.update(trial_vectors=trials, key=key)

    def tell(self, state, trial_fitness):
        B = self.batch_size
        tf = trial_fitness.reshape(3, B)
        best3 = torch.argmin(tf, 0)
        g = best3 * B + torch.arange(B, device=tf.device)
        cur = self._cur(state)
        pop, fit, _ = C.greedy_replace(state.population, state.fitness, state.trial_vectors[g], trial_fitness[g], cur,
                                       strict=False)
        return state.update(population=pop, fitness=fit, best_index=torch.argmin(fit),
                            start_index=(state.start_index + B) % self.pop_size)
