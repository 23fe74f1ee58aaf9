"""Comprehensive-learning PSO (Liang et al. 2006; reference ``pso_variants/clpso.py:17-121``)."""
from __future__ import annotations

import torch

from ....core import Algorithm, State
from ....ops import random as rnd
from ....parallel.dim_sharded import ColumnSeparable
from .utils import init_swarm, min_by


class CLPSO(ColumnSeparable, Algorithm):
    # decision-axis state sharding (P2): positions, velocities and the personal / global bests
    # are column blocks; exemplar choice and the best updates use the replicated fitness only
    column_separable = True
    dim_fields = ("population", "velocity", "pbest_position", "gbest_position")

    def __init__(self, lb, ub, pop_size, inertia_weight, const_coefficient, learning_probability):
        super().__init__()
        self.dim = lb.shape[0]
        self.lb, self.ub, self.pop_size = lb, ub, pop_size
        self.w, self.c = inertia_weight, const_coefficient
        self.P_c = torch.as_tensor(learning_probability, dtype=torch.float32, device=lb.device).expand(pop_size)

    def setup(self, key):
        state_key, kp, kv = rnd.split(key, 3)
        pop, vel = init_swarm(kp, kv, self.pop_size, self.lb, self.ub)
        dev = pop.device
        return State(population=pop, velocity=vel, pbest_position=pop, pbest_fitness=torch.full((self.pop_size,), float("inf"), device=dev),
                     gbest_position=pop[0], gbest_fitness=torch.full((1,), float("inf"), device=dev), key=state_key)

    def ask(self, state):
        return state.population, state

    def tell(self, state, fitness):
        key, k_coef, k1, k2, k_rand = rnd.split(state.key, 5)
        dev = fitness.device
        N, d = self.pop_size, self.dim
        coef = self.uniform_cols(k_coef, N, dev)
        better = state.pbest_fitness > fitness
        pbest_position = torch.where(better[:, None], state.population, state.pbest_position)
        pbest_fitness = torch.minimum(state.pbest_fitness, fitness)
        gpos, gfit = min_by([state.gbest_position[None, :], state.population], [state.gbest_fitness, fitness])
        r1 = torch.floor(rnd.uniform(k1, (N,), minval=0.0, maxval=float(N)).to(dev)).long().clamp(max=N - 1)
        r2 = torch.floor(rnd.uniform(k2, (N,), minval=0.0, maxval=float(N)).to(dev)).long().clamp(max=N - 1)
        learn = torch.where(pbest_fitness[r1] < pbest_fitness[r2], r1, r2)
        learning_pbest = state.pbest_position[learn]
        rp = rnd.uniform(k_rand, (N,)).to(dev)
        pbest = torch.where((rp < self.P_c)[:, None], learning_pbest, state.pbest_position)
        velocity = self.w * state.velocity + self.c * coef * (pbest - state.population)
        population = torch.clamp(state.population + velocity, self.col_vec(self.lb), self.col_vec(self.ub))
        return state.update(population=population, velocity=velocity, pbest_position=pbest_position, pbest_fitness=pbest_fitness,
                            gbest_position=gpos, gbest_fitness=gfit.reshape(1), key=key)
