"""EPSDE — ensemble of mutation strategies and parameters (reference ``de_variants/epsde.py:30-194``).

Each individual carries a parameter vector [strategy code (4), F, CR] drawn from
{rand/1/bin, best/2/bin, current-to-rand/1/bin} × F ∈ {0.4..0.9} × CR ∈ {0.1..0.9}.
Successful vectors persist; after a failure the individual re-draws, either a
random new vector or (with probability 1/2) the last successful vector of its slot.
"""
from __future__ import annotations

import torch

from ....core import Algorithm
from ....ops import random as rnd
from . import common as C

F_POOL = torch.arange(4, 10, dtype=torch.float32) / 10.0
CR_POOL = torch.arange(1, 10, dtype=torch.float32) / 10.0
EPSDE_STRATEGIES = torch.tensor([C.rand_1_bin, C.best_2_bin, C.current2rand_1_bin], dtype=torch.float32)


def random_params(ks, kf, kc, n, device):
    s = C.dconst(EPSDE_STRATEGIES, device)[rnd.randint(ks, (n,), 0, 3).to(device)]
    f = C.dconst(F_POOL, device)[rnd.randint(kf, (n,), 0, 6).to(device)]
    c = C.dconst(CR_POOL, device)[rnd.randint(kc, (n,), 0, 9).to(device)]
    return torch.cat([s, f[:, None], c[:, None]], 1)


def param_trials(key, state, params, cur, diff_padding_num, p, lb, ub):
    strat = params[:, :4].to(torch.int64)
    return C.generate_trials(key, state.population, state.fitness, state.best_index, cur, strat, params[:, 4], params[:, 5],
                             diff_padding_num, lb, ub, p=p)[0]


class EPSDE(Algorithm):
    def __init__(self, lb, ub, pop_size=100, diff_padding_num=5, differential_weight=None, cross_probability=None, p=0.05):
        super().__init__()
        self.dim = lb.shape[0]
        self.lb, self.ub = lb, ub
        self.pop_size = pop_size
        self.diff_padding_num = diff_padding_num
        self.p = p

    def setup(self, key):
        state_key, init_key, ks, kf, kc = rnd.split(key, 5)
        pop = C.init_population(init_key, self.pop_size, self.lb, self.ub)
        dev = pop.device
        pv = random_params(ks, kf, kc, self.pop_size, dev)
        return C.base_state(state_key, pop, trial_vectors=torch.zeros_like(pop), param_vect=pv, S_param_vect=pv.clone(),
                            compare=torch.ones(self.pop_size, dtype=torch.bool, device=dev))

    def ask(self, state):
        key, k_trial, ks, k_renew, kf, kc = rnd.split(state.key, 6)
        dev = state.population.device
        N = self.pop_size
        rand_pv = random_params(ks, kf, kc, N, dev)
        renew = rnd.randint(k_renew, (N,), 0, 2).to(dev).bool()
        renewed = torch.where(renew[:, None], state.S_param_vect, rand_pv)
        pv = torch.where(state.compare[:, None], state.param_vect, renewed)
        trials = param_trials(k_trial, state, pv, torch.arange(N, device=dev), self.diff_padding_num, self.p, self.lb, self.ub)
        return trials, state.update(trial_vectors=trials, key=key, param_vect=pv)

    def tell(self, state, trial_fitness):
        pop, fit, ok = C.greedy_replace(state.population, state.fitness, state.trial_vectors, trial_fitness, strict=True)
        S = torch.where(ok[:, None], state.param_vect, state.S_param_vect)
        return state.update(population=pop, fitness=fit, best_index=torch.argmin(fit), S_param_vect=S, compare=ok)
