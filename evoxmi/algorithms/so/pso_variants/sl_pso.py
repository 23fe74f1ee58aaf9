"""Social-learning PSO with Gaussian / uniform demonstrator choice
(Cheng & Jin 2015; reference ``pso_variants/sl_pso_gs.py:17-94``, ``sl_pso_us.py:18-94``)."""
from __future__ import annotations

import math

import torch

from ....core import Algorithm, State
from ....ops import random as rnd
from .utils import init_swarm, min_by


class _SLPSO(Algorithm):
    def __init__(self, lb, ub, pop_size, social_influence_factor, demonstrator_choice_factor):
        super().__init__()
        self.dim = lb.shape[0]
        self.lb, self.ub, self.pop_size = lb, ub, pop_size
        self.social_influence_factor = social_influence_factor
        self.demonstrator_choice_factor = demonstrator_choice_factor

    def setup(self, key):
        state_key, kp, kv = rnd.split(key, 3)
        pop, vel = init_swarm(kp, kv, self.pop_size, self.lb, self.ub)
        return State(population=pop, velocity=vel, global_best_location=pop[0],
                     global_best_fitness=torch.full((1,), float("inf"), device=pop.device), key=state_key)

    def ask(self, state):
        return state.population, state

    def _index_k(self, key, device):
        raise NotImplementedError

    def tell(self, state, fitness):
        key, k1, k2, k3, k_demo = rnd.split(state.key, 5)
        dev = fitness.device
        N, d = self.pop_size, self.dim
        r1, r2, r3 = (rnd.uniform(k, (N, d)).to(dev) for k in (k1, k2, k3))
        gpos, gfit = min_by([state.global_best_location[None, :], state.population], [state.global_best_fitness, fitness])
        ranked = state.population[torch.argsort(-fitness, stable=True)]
        X_k = ranked[self._index_k(k_demo, dev)]
        X_avg = state.population.mean(0)
        velocity = r1 * state.velocity + r2 * (X_k - state.population) + r3 * self.social_influence_factor * (X_avg - state.population)
        population = torch.clamp(state.population + velocity, self.lb, self.ub)
        return state.update(population=population, velocity=velocity, global_best_location=gpos, global_best_fitness=gfit.reshape(1), key=key)


class SLPSOGS(_SLPSO):
    def _index_k(self, key, device):
        N = self.pop_size
        sigma = self.demonstrator_choice_factor * (N - (torch.arange(N, device=device) + 1))
        nd = sigma * (-torch.abs(rnd.normal(key, (N,)).to(device))) + N
        return torch.floor(torch.clamp(nd, 1, N)).long() - 1


class SLPSOUS(_SLPSO):
    def _index_k(self, key, device):
        N = self.pop_size
        q = torch.clamp(N - torch.ceil(self.demonstrator_choice_factor * (N - (torch.arange(N, device=device) + 1) - 1)), 1, N)
        u = rnd.uniform(key, (N,)).to(device) * (N + 1 - q) + q
        return (torch.floor(u).long() - 1).clamp(0, N - 1)
