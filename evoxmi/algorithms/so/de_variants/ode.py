"""Opposition-based DE (reference ``algorithms/so/de_variants/ode.py:18-187``).

Odd generations (the counter starts at 1) propose the opposite points
``lb + ub − base`` (no crossover, no clip — as in the reference's ``_ask_one_odd``);
even generations do a classic DE step.  Both branches are computed and selected on
the device-side counter so the step stays capturable in a hipGraph.  Rows are
processed in circular batches of ``batch_size`` starting at ``start_index``.
"""
from __future__ import annotations

import torch

from ....core import Algorithm
from ....ops import random as rnd
from . import common as C
from .de import DE


class ODE(DE):
    # decision-axis state sharding: the opposite point lb + ub − base is per column too
    column_separable = True

    def __init__(self, lb, ub, pop_size, base_vector="rand", num_difference_vectors=1, differential_weight=0.5,
                 cross_probability=0.9, batch_size=100, replace=False, mean=None, stdvar=None):
        super().__init__(lb, ub, pop_size, base_vector, num_difference_vectors, differential_weight, cross_probability,
                         batch_size, replace, mean, stdvar)
        self.batch_size = min(batch_size, pop_size)

    def setup(self, key):
        st = super().setup(key)
        dev = st.population.device
        return st.update(trial_vectors=torch.empty((self.batch_size, self.dim), device=dev),
                         start_index=C.scalar(0, dev, torch.int64), counter=C.scalar(1, dev, torch.int64))

    def _cur(self, state):
        dev = state.population.device
        return (torch.arange(self.batch_size, device=dev) + state.start_index) % self.pop_size

    def ask(self, state):
        key, r_key = rnd.split(state.key)
        pop = state.population
        N = pop.shape[0]
        cur = self._cur(state)
        k_ch, k_tr = rnd.split(r_key)
        ch = self._choices(k_ch, N, cur)
        b = C.BEST if self.base_vector == "best" else C.RAND
        strat = (b, b, self.num_difference_vectors, C.BIN)
        # column block of a decision-axis-sharded state (dim_shard), else all columns
        c0, own, d = self.cols()
        lb, ub = self.lb[c0 : c0 + own], self.ub[c0 : c0 + own]
        de_trials, _ = C.generate_trials(k_tr, pop, state.fitness, state.best_index, cur, strat, self.differential_weight,
                                         self.cross_probability, 0, lb, ub, choices=ch, cols=(c0, d))
        base = pop.index_select(0, state.best_index.reshape(1)).expand(cur.shape[0], -1) if self.base_vector == "best" else pop[ch[:, 0]]
        opposite = ub + lb - base
        trials = torch.where(state.counter % 2 == 0, de_trials, opposite)
        return trials, state.update(trial_vectors=trials, key=key)

    def tell(self, state, trial_fitness):
        cur = self._cur(state)
        pop, fit, _ = C.greedy_replace(state.population, state.fitness, state.trial_vectors, trial_fitness, cur, strict=True)
        return state.update(population=pop, fitness=fit, best_index=torch.argmin(fit),
                            start_index=(state.start_index + self.batch_size) % self.pop_size, counter=state.counter + 1)
