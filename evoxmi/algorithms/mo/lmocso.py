"""LMOCSO — competitive swarm for large-scale MOPs (Tian et al. 2020; reference ``algorithms/mo/lmocso.py:44-184``).

Losers of random pairings (compared by shift-based density) learn from winners with
a two-step velocity update, polynomial mutation, RVEA's APD environmental selection.
"""
from __future__ import annotations

import torch

from ...core import State
from ...operators import selection
from ...operators.sampling import UniformSampling
from ...ops import random as rnd
from .common import MOAlgorithm


def cal_fitness(obj):
    n = obj.shape[0]
    f = (obj - obj.min(0).values) / (obj.max(0).values - obj.min(0).values)
    d = torch.sqrt((torch.clamp(f[None, :, :] - f[:, None, :], min=0) ** 2).sum(-1))  # ‖f_i − max(f_j, f_i)‖
    return d.masked_fill(torch.eye(n, dtype=torch.bool, device=obj.device), float("inf")).min(1).values


class LMOCSO(MOAlgorithm):
    def __init__(self, n_objs, lb, ub, pop_size, alpha=2, max_gen=100, selection_op=None, mutation_op=None):
        super().__init__(lb, ub, n_objs, pop_size, mutation_op)
        self.alpha, self.max_gen = alpha, max_gen
        self.selection = selection_op if selection_op is not None else selection.ReferenceVectorGuided()
        self.sampling = UniformSampling(pop_size, n_objs)

    def setup(self, key):
        state_key, init_key, vkey = rnd.split(key, 3)
        v = self.sampling(vkey)[0].to(self.lb.device)
        self.pop_size = v.shape[0]
        pop = self._init_pop(init_key)
        return State(population=pop, next_generation=pop, fitness=torch.full((self.pop_size, self.n_objs), float("inf"), device=pop.device),
                     velocity=torch.zeros((self.pop_size // 2 * 2, self.dim), device=pop.device), key=state_key, reference_vector=v,
                     gen=torch.zeros((), dtype=torch.int64, device=pop.device))

    def ask(self, state):
        key, k_mate, k_pair, k0, k1, mut_key = rnd.split(state.key, 6)
        dev = state.population.device
        N, h = self.pop_size, self.pop_size // 2
        valid = ~torch.isnan(state.population).all(1)
        order = torch.argsort((~valid).to(torch.int64), stable=True)
        r = torch.floor(rnd.uniform(k_mate, (N,)).to(dev) * valid.sum().clamp(min=1)).long()
        population = state.population[order[r]]
        perm = rnd.permutation(k_pair, h * 2).to(dev).reshape(2, h)
        sde = cal_fitness(torch.nan_to_num(state.fitness, nan=float("inf")))
        m = sde[perm[0]] > sde[perm[1]]
        winner, loser = torch.where(m, perm[0], perm[1]), torch.where(m, perm[1], perm[0])
        r0, r1 = rnd.uniform(k0, (h, self.dim)).to(dev), rnd.uniform(k1, (h, self.dim)).to(dev)
        v_l = state.velocity[loser]
        off_v = r0 * v_l + r1 * (population[winner] - population[loser])
        new_l = torch.clamp(population[loser] + off_v + r0 * (off_v - v_l), self.lb, self.ub)
        new_pop = population.index_copy(0, loser, new_l)
        vel = state.velocity.index_copy(0, loser, off_v)
        off = self.mutation(mut_key, new_pop)
        return off, state.update(next_generation=off, velocity=vel, key=key)

    def tell(self, state, fitness):
        gen = state.gen + 1
        surv, surv_fit = self.selection(torch.cat([state.population, state.next_generation]), torch.cat([state.fitness, fitness]),
                                        state.reference_vector, (gen.to(torch.float32) / self.max_gen) ** self.alpha)
        return state.update(population=surv, fitness=surv_fit, gen=gen)
