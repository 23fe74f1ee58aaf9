"""Dynamic multi-swarm PSO with elite learning (reference ``pso_variants/dms_pso_el.py:17-338``).

Strategy 1 (first 90 % of ``max_iteration``): dynamic sub-swarms learn from their
local best, the following swarm from "rbest" elites, with regrouping (sort, shuffle
the best part into sub-swarms) every ``regrouped_iteration_num`` iterations.
Strategy 2: global-best PSO.  Both strategies (and the regroup) are evaluated and
selected on the device-side iteration counter, so a generation stays one capturable
hipGraph.
"""
from __future__ import annotations

import torch

from ....core import Algorithm, State
from ....ops import random as rnd
from .utils import init_swarm


class DMSPSOEL(Algorithm):
    def __init__(self, lb, ub, dynamic_sub_swarm_size, dynamic_sub_swarms_num, following_sub_swarm_size, regrouped_iteration_num,
                 max_iteration, inertia_weight, pbest_coefficient, lbest_coefficient, rbest_coefficient, gbest_coefficient):
        super().__init__()
        self.dim = lb.shape[0]
        self.lb, self.ub = lb, ub
        self.S, self.M, self.F = dynamic_sub_swarm_size, dynamic_sub_swarms_num, following_sub_swarm_size
        self.pop_size = self.S * self.M + self.F
        self.R = regrouped_iteration_num
        self.max_iteration = max_iteration
        self.w = inertia_weight
        self.c_pbest, self.c_lbest, self.c_rbest, self.c_gbest = pbest_coefficient, lbest_coefficient, rbest_coefficient, gbest_coefficient

    def setup(self, key):
        state_key, kp, kv = rnd.split(key, 3)
        pop, vel = init_swarm(kp, kv, self.pop_size, self.lb, self.ub)
        dev = pop.device
        return State(iteration=torch.zeros((), dtype=torch.int64, device=dev), population=pop, velocity=vel, pbest_position=pop,
                     pbest_fitness=torch.full((self.pop_size,), float("inf"), device=dev),
                     lbest_position=pop[: self.S * self.M].reshape(self.M, self.S, self.dim)[:, 0, :].clone(),
                     lbest_fitness=torch.full((self.M,), float("inf"), device=dev),
                     rbest_index=torch.zeros(self.F, dtype=torch.int64, device=dev), gbest_position=torch.zeros(self.dim, device=dev),
                     gbest_fitness=torch.tensor(float("inf"), device=dev), key=state_key)

    def ask(self, state):
        return state.population, state

    def _regroup(self, state, fitness):
        SM = self.S * self.M
        order = torch.argsort(fitness, stable=True)
        state_key, shuffle_key = rnd.split(state.key)
        dyn = order[:SM][rnd.permutation(shuffle_key, SM).to(order.device)]
        idx = torch.cat([dyn, order[SM:]])
        # the F best of the dynamic part (cycled when F > S·M, where the reference's slice is short)
        rbest_index = torch.argsort(fitness[:SM], stable=True)[torch.arange(self.F, device=fitness.device) % SM]
        return dict(population=state.population[idx], velocity=state.velocity[idx], pbest_position=state.pbest_position[idx],
                    pbest_fitness=state.pbest_fitness[idx], rbest_index=rbest_index, key=state_key)

    def tell(self, state, fitness):
        SM, S, M, d = self.S * self.M, self.S, self.M, self.dim
        # strategy 1 (with conditional regroup, reference :93-99)
        do_regroup = (state.iteration % self.R) == 0
        rg = self._regroup(state, fitness)
        pick = lambda name: torch.where(do_regroup, rg[name], state[name]) if rg[name].dim() == 0 else \
            torch.where(do_regroup.reshape((1,) * rg[name].dim()), rg[name], state[name])
        pop, vel = pick("population"), pick("velocity")
        pb_pos, pb_fit, rbest_index, key1 = pick("pbest_position"), pick("pbest_fitness"), pick("rbest_index"), pick("key")
        state_key, k_pb, k_lb, k_rb = rnd.split(key1, 4)
        better = pb_fit > fitness
        pb_pos = torch.where(better[:, None], pop, pb_pos)
        pb_fit = torch.minimum(pb_fit, fitness)
        dyn_pos = pop[:SM].reshape(M, S, d)
        dyn_fit = fitness[:SM].reshape(M, S)
        lbest_fitness, lbest_idx = dyn_fit.min(1)
        lbest_position = dyn_pos[torch.arange(M, device=pop.device), lbest_idx]
        rbest_position = pop[rbest_index]
        rand_pb = rnd.uniform(k_pb, (self.pop_size, d)).to(pop.device)
        rand_lb = rnd.uniform(k_lb, (M, S, d)).to(pop.device)
        dyn_v = (self.w * vel[:SM].reshape(M, S, d) + self.c_pbest * rand_pb[:SM].reshape(M, S, d) * (pb_pos[:SM].reshape(M, S, d) - dyn_pos)
                 + self.c_lbest * rand_lb * (lbest_position[:, None, :] - dyn_pos))
        rand_rb = rnd.uniform(k_rb, (self.F, d)).to(pop.device)
        fol_pos = pop[SM:]
        fol_v = self.w * vel[SM:] + self.c_pbest * rand_pb[SM:] * (pb_pos[SM:] - fol_pos) + self.c_rbest * rand_rb * (rbest_position - fol_pos)
        v1 = torch.cat([dyn_v.reshape(SM, d), fol_v])
        s1 = dict(population=torch.clamp(pop + v1, self.lb, self.ub), velocity=v1, pbest_position=pb_pos, pbest_fitness=pb_fit,
                  lbest_position=lbest_position, lbest_fitness=lbest_fitness, rbest_index=rbest_index,
                  gbest_position=state.gbest_position, gbest_fitness=state.gbest_fitness, key=state_key)
        # strategy 2: global-best PSO (reference :275-338)
        k2s, k2p, k2g = rnd.split(state.key, 3)
        better2 = state.pbest_fitness > fitness
        pb_pos2 = torch.where(better2[:, None], state.population, state.pbest_position)
        pb_fit2 = torch.minimum(state.pbest_fitness, fitness)
        gi = torch.argmin(pb_fit2)
        g_pos = pb_pos2.index_select(0, gi.reshape(1))[0]
        g_fit = pb_fit2.min()
        v2 = (self.w * state.velocity + self.c_pbest * rnd.uniform(k2p, (self.pop_size, d)).to(pop.device) * (pb_pos2 - state.population)
              + self.c_gbest * rnd.uniform(k2g, (self.pop_size, d)).to(pop.device) * (g_pos - state.population))
        s2 = dict(population=torch.clamp(state.population + v2, self.lb, self.ub), velocity=v2, pbest_position=pb_pos2,
                  pbest_fitness=pb_fit2, lbest_position=state.lbest_position, lbest_fitness=state.lbest_fitness,
                  rbest_index=state.rbest_index, gbest_position=g_pos, gbest_fitness=g_fit, key=k2s)
        first = state.iteration < 0.9 * self.max_iteration
        out = {k: torch.where(first.reshape((1,) * s1[k].dim()) if s1[k].dim() else first, s1[k], s2[k]) for k in s1}
        return state.update(iteration=state.iteration + 1, **out)
