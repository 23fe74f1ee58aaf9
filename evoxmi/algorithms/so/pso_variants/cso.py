"""Competitive swarm optimiser (Cheng & Jin 2015; reference ``pso_variants/cso.py:26-103``).

Random pairing; each loser learns from its winner and (φ-weighted) from the swarm
centre; only the N/2 losers are re-evaluated per generation (``init_ask`` /
``init_tell`` evaluate everyone once).
"""
from __future__ import annotations

import torch

from ....core import Algorithm, State
from ....ops import random as rnd
from ....parallel.dim_sharded import ColumnSeparable


class CSO(ColumnSeparable, Algorithm):
    # decision-axis state sharding (P2): positions and velocities are column blocks, the
    # pairing comes from the replicated fitness, the learning coefficients are drawn per
    # global column and the swarm centre is a per-column mean
    column_separable = True
    dim_fields = ("population", "velocity")

    def __init__(self, lb, ub, pop_size, phi=0.0, mean=None, stdev=None):
        super().__init__()
        self.lb, self.ub, self.pop_size, self.phi = lb, ub, pop_size, phi
        self.mean, self.stdev = mean, stdev
        self.dim = lb.shape[0]

    def setup(self, key):
        state_key, init_key = rnd.split(key)
        dev = self.lb.device
        if self.mean is not None and self.stdev is not None:
            pop = torch.clamp(self.mean + self.stdev * rnd.normal(init_key, (self.pop_size, self.dim)).to(dev), self.lb, self.ub)
        else:
            pop = rnd.uniform(init_key, (self.pop_size, self.dim)).to(dev) * (self.ub - self.lb) + self.lb
        return State(population=pop, fitness=torch.full((self.pop_size,), float("inf"), device=dev),
                     velocity=torch.zeros_like(pop), students=torch.zeros(self.pop_size // 2, dtype=torch.int64, device=dev),
                     key=state_key)

    def init_ask(self, state):
        return state.population, state

    def init_tell(self, state, fitness):
        return state.update(fitness=fitness)

    def ask(self, state):
        key, k_pair, k1, k2, k3 = rnd.split(state.key, 5)
        dev = state.population.device
        h = self.pop_size // 2
        perm = rnd.permutation(k_pair, self.pop_size).to(dev)[: 2 * h].reshape(2, h)
        mask = state.fitness[perm[0]] < state.fitness[perm[1]]
        teachers = torch.where(mask, perm[0], perm[1])
        students = torch.where(mask, perm[1], perm[0])
        l1, l2, l3 = (self.uniform_cols(k, h, dev) for k in (k1, k2, k3))
        center = state.population.mean(0)
        ps = state.population[students]
        v = l1 * state.velocity[students] + l2 * (state.population[teachers] - ps) + self.phi * l3 * (center - ps)
        cand = torch.clamp(ps + v, self.col_vec(self.lb), self.col_vec(self.ub))
        pop = state.population.index_copy(0, students, cand)
        vel = state.velocity.index_copy(0, students, v)
        return cand, state.update(population=pop, velocity=vel, students=students, key=key)

    def tell(self, state, fitness):
        return state.update(fitness=state.fitness.index_copy(0, state.students, fitness))
