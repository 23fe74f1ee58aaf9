"""FSPSO — GA/PSO hybrid (reference ``pso_variants/fs_pso.py:20-159``; not exported there).

The better half is updated by PSO; the other half is refilled by binary-tournament
selection from the elite plus uniform-offset mutation.
"""
from __future__ import annotations

import torch

from ....core import Algorithm, State
from ....ops import random as rnd
from .utils import init_swarm, min_by


class FSPSO(Algorithm):
    def __init__(self, lb, ub, pop_size, inertia_weight=0.6, cognitive_coefficient=2.5, social_coefficient=0.8, mean=None, stdev=None,
                 mutate_rate=0.01):
        super().__init__()
        self.dim = lb.shape[0]
        self.lb, self.ub, self.pop_size = lb, ub, pop_size
        self.w, self.phi_p, self.phi_g = inertia_weight, cognitive_coefficient, social_coefficient
        self.mean, self.stdev, self.mutate_rate = mean, stdev, mutate_rate

    def setup(self, key):
        state_key, kp, kv = rnd.split(key, 3)
        pop, vel = init_swarm(kp, kv, self.pop_size, self.lb, self.ub, self.mean, self.stdev)
        return State(population=pop, velocity=vel, local_best_location=pop,
                     local_best_fitness=torch.full((self.pop_size,), float("inf"), device=pop.device), global_best_location=pop[0],
                     global_best_fitness=torch.full((1,), float("inf"), device=pop.device), key=state_key)

    def ask(self, state):
        return state.population, state

    def tell(self, state, fitness):
        key, k_rg, k_rp, k_tn, k_mu, k_ma = rnd.split(state.key, 6)
        dev = fitness.device
        N, d, h = self.pop_size, self.dim, self.pop_size // 2
        elite = torch.argsort(fitness, stable=True)[:h]
        e_pop, e_vel, e_fit = state.population[elite], state.velocity[elite], fitness[elite]
        e_lbl, e_lbf = state.local_best_location[elite], state.local_best_fitness[elite]
        rg, rp = rnd.uniform(k_rg, (h, d)).to(dev), rnd.uniform(k_rp, (h, d)).to(dev)
        better = e_lbf > e_fit
        lbl = torch.where(better[:, None], e_pop, e_lbl)
        lbf = torch.minimum(e_lbf, e_fit)
        gpos, gfit = min_by([state.global_best_location[None, :], e_pop], [state.global_best_fitness, e_fit])
        new_v = self.w * e_vel + self.phi_p * rp * (e_lbl - e_pop) + self.phi_g * rg * (gpos - e_pop)
        new_e = torch.clamp(e_pop + new_v, self.lb, self.ub)
        n_off = N - h
        # the reference draws both tournament columns with the same key (fs_pso.py:111-120),
        # so every "tournament" compares a contestant with itself; two keys here
        kt1, kt2 = rnd.split(k_tn)
        t1 = rnd.randint(kt1, (n_off,), 0, h).to(dev)
        t2 = rnd.randint(kt2, (n_off,), 0, h).to(dev)
        pool = torch.where(e_fit[t1] < e_fit[t2], t1, t2)
        parents, off_v = e_pop[pool], e_vel[pool]
        offset = (rnd.uniform(k_mu, (n_off, d)).to(dev) * 2 - 1) * (self.ub - self.lb)
        mask = rnd.uniform(k_ma, (n_off, d)).to(dev) < self.mutate_rate
        off = torch.clamp(parents + torch.where(mask, offset, torch.zeros_like(offset)), self.lb, self.ub)
        return state.update(population=torch.cat([new_e, off]), velocity=torch.cat([new_v, off_v]),
                            local_best_location=torch.cat([lbl, off]),
                            local_best_fitness=torch.cat([lbf, torch.full((n_off,), float("inf"), device=dev)]),
                            global_best_location=gpos, global_best_fitness=gfit.reshape(1), key=key)
