"""Classic DE (reference ``algorithms/so/de_variants/de.py:11-168``).

rand/1 or best/1 base with ``num_difference_vectors`` difference pairs, binomial
crossover with a forced j_rand, clip, greedy one-to-one replacement.  The
reference's ``batch_size`` argument is ignored there (``:40``, batch = pop_size);
the same here.  Trial generation is the fused ``de_trial`` HIP kernel.
"""
from __future__ import annotations

import torch

from ....core import Algorithm, State
from ....ops import random as rnd
from ....parallel.dim_sharded import ColumnSeparable
from . import common as C


class DE(ColumnSeparable, Algorithm):
    def __init__(self, lb, ub, pop_size, base_vector="rand", num_difference_vectors=1, differential_weight=0.5,
                 cross_probability=0.9, batch_size=100, replace=False, mean=None, stdvar=None):
        super().__init__()
        assert torch.all(lb < ub)
        assert pop_size >= 4
        assert 0 < cross_probability <= 1
        assert base_vector in ("rand", "best")
        self.num_difference_vectors = num_difference_vectors
        self.dim = lb.shape[0]
        self.lb, self.ub = lb, ub
        self.pop_size = pop_size
        self.base_vector = base_vector
        self.batch_size = pop_size
        self.replace = replace
        self.cross_probability = cross_probability
        self.differential_weight = differential_weight
        self.mean, self.stdvar = mean, stdvar

    def setup(self, key):
        state_key, init_key = rnd.split(key)
        pop = C.init_population(init_key, self.pop_size, self.lb, self.ub, self.mean, self.stdvar)
        return C.base_state(state_key, pop, trial_vectors=torch.empty_like(pop))

    def _choices(self, key, N, cur):
        k = 2 * self.num_difference_vectors + 1
        if self.replace:
            ch = rnd.randint(key, (cur.shape[0], k), 0, N).to(cur.device)
        else:
            ch = C.sample_distinct(key, cur.shape[0], k, N, None, cur.device)
        return C._remap_self(ch, cur, N)

    # -- decision-axis state sharding (P2): mutation, crossover and the greedy replacement are
    # column-separable given the replicated per-row draws (difference rows, j_rand) and the
    # replicated fitness, so a rank keeps only its column block of population and trials
    # opt-in flag (parallel.dim_sharded.algorithm_column_separable): a subclass with its own
    # ask / tell must declare itself column-separable again
    column_separable = True
    dim_fields = ("population", "trial_vectors")

    def _trials(self, state, key):
        pop = state.population
        N = pop.shape[0]
        k_ch, k_tr = rnd.split(key)
        cur = torch.arange(N, device=pop.device)
        b = C.BEST if self.base_vector == "best" else C.RAND
        strat = (b, b, self.num_difference_vectors, C.BIN)
        c0, own, d = self.cols()
        trials, _ = C.generate_trials(k_tr, pop, state.fitness, state.best_index, cur, strat, self.differential_weight,
                                      self.cross_probability, 0, self.lb[c0 : c0 + own], self.ub[c0 : c0 + own],
                                      choices=self._choices(k_ch, N, cur), cols=(c0, d))
        return trials

    def ask(self, state):
        key, r_key = rnd.split(state.key)
        trials = self._trials(state, r_key)
        return trials, state.update(trial_vectors=trials, key=key)

    def tell(self, state, trial_fitness):
        pop, fit, _ = C.greedy_replace(state.population, state.fitness, state.trial_vectors, trial_fitness, strict=True)
        return state.update(population=pop, fitness=fit, best_index=torch.argmin(fit))
