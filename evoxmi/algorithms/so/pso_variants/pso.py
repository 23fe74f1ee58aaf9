"""Particle Swarm Optimisation (reference ``algorithms/so/pso_variants/pso.py:19-108``).

``ask`` returns the stored swarm; ``tell`` updates personal bests, the global best
(``min_by`` over [gbest; swarm]) and the velocity
``v ← w v + φp rp (pbest − x) + φg rg (gbest − x)``, then clips to the box.
On a GPU the whole ``tell`` is a single fused HIP kernel (K7: Philox draws for
``rp``/``rg`` generated in-register, pbest select, velocity/position update and
clip in one pass over the (N, d) arrays) after a device-side argmin.
"""
from __future__ import annotations

import torch

from ....core import Algorithm, State
from ....ops import random as rnd
from ....ops import pso as pso_ops
from ....parallel.dim_sharded import ColumnSeparable


class PSO(ColumnSeparable, Algorithm):
    def __init__(self, lb, ub, pop_size, inertia_weight=0.6, cognitive_coefficient=2.5, social_coefficient=0.8, mean=None, stdev=None):
        super().__init__()
        self.dim = lb.shape[0]
        self.lb = lb
        self.ub = ub
        self.pop_size = pop_size
        self.w = inertia_weight
        self.phi_p = cognitive_coefficient
        self.phi_g = social_coefficient
        self.mean = mean
        self.stdev = stdev

    def setup(self, key):
        state_key, init_pop_key, init_v_key = rnd.split(key, 3)
        dev = self.lb.device
        lb, ub = self.lb, self.ub
        if self.mean is not None and self.stdev is not None:
            population = self.stdev * rnd.normal(init_pop_key, (self.pop_size, self.dim)).to(dev)
            population = torch.clamp(population, lb, ub)
            velocity = self.stdev * rnd.normal(init_v_key, (self.pop_size, self.dim)).to(dev)
        else:
            length = ub - lb
            population = rnd.uniform(init_pop_key, (self.pop_size, self.dim)).to(dev) * length + lb
            velocity = rnd.uniform(init_v_key, (self.pop_size, self.dim)).to(dev) * length * 2 - length
        return State(
            population=population,
            velocity=velocity,
            local_best_location=population,
            local_best_fitness=torch.full((self.pop_size,), float("inf"), device=dev),
            global_best_location=population[0],
            global_best_fitness=torch.tensor([float("inf")], device=dev),
            key=state_key,
        )

    def ask(self, state):
        return state.population, state

    # -- decision-axis state sharding (P2, StdWorkflow.enable_multi_devices): every (N, d) / (d,)
    # field is column-separable in the tell (the only row coupling is through the replicated
    # fitness), so a rank keeps only its column block and nothing but the evaluation's per-row
    # terms crosses the ranks
    column_separable = True
    dim_fields = ("population", "velocity", "local_best_location", "global_best_location")

    def tell(self, state, fitness):
        key, rg_key, rp_key = rnd.split(state.key, 3)
        # global best over [gbest; swarm] — device argmin, no host sync
        i = torch.argmin(fitness)
        cand_f = fitness[i].reshape(1)
        better = cand_f < state.global_best_fitness
        global_best_fitness = torch.where(better, cand_f, state.global_best_fitness)
        global_best_location = torch.where(better, state.population[i], state.global_best_location)
        c0, own, d = self.cols()
        pos, vel, lbl, lbf = pso_ops.pso_update(
            state.population, state.velocity, state.local_best_location, state.local_best_fitness, fitness,
            global_best_location, rp_key, rg_key, self.w, self.phi_p, self.phi_g, self.lb[c0 : c0 + own], self.ub[c0 : c0 + own],
            col0=c0, d_total=d,
        )
        return state.update(
            population=pos,
            velocity=vel,
            local_best_location=lbl,
            local_best_fitness=lbf,
            global_best_location=global_best_location,
            global_best_fitness=global_best_fitness,
            key=key,
        )
