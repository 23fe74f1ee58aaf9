"""EAG-MOEA/D — external-archive-guided MOEA/D (Cai et al. 2015; reference ``algorithms/mo/eagmoead.py:43-212``).

An internal MOEA/D population (weighted-sum decomposition, sequential neighbourhood
replacement run as one wave-level kernel) produces offspring; an external archive is
maintained by NSGA-II selection; subproblems whose offspring enter the archive get
more computing resource (success memory over the last LGs generations drives a
roulette wheel).  The reference's success bookkeeping writes column
``gen % LGs + 1`` (out of range for the last column, clamped by JAX) after a
padded ``where``; here the success count of each subproblem is stored in column
``gen % LGs``.
"""
from __future__ import annotations

import math

import torch

from ...core import State
from ...operators import crossover, selection
from ...operators.sampling import LatinHypercubeSampling
from ...ops import mo as mo_ops
from ...ops import random as rnd
from .common import MOAlgorithm, nsga2_select, weights_and_neighbours


class EAGMOEAD(MOAlgorithm):
    def __init__(self, lb, ub, n_objs, pop_size, LGs=8, selection_op=None, mutation_op=None, crossover_op=None):
        super().__init__(lb, ub, n_objs, pop_size, mutation_op, crossover_op if crossover_op is not None else crossover.SimulatedBinary(type=2))
        self.LGs = LGs
        self.T = math.ceil(pop_size / 10)
        self.selection = selection_op if selection_op is not None else selection.RouletteWheelSelection(pop_size)
        self.sample = LatinHypercubeSampling(pop_size, n_objs)

    def setup(self, key):
        key, k1, k2 = rnd.split(key, 3)
        pop = self._init_pop(k1)
        dev = pop.device
        N = self.pop_size
        w = self.sample(k2)[0].to(dev)
        f = torch.zeros((N, self.n_objs), device=dev)
        return State(population=pop, fitness=f, inner_pop=pop.clone(), inner_obj=f.clone(), next_generation=pop, weight_vector=w,
                     B=weights_and_neighbours(w, self.T), s=torch.zeros((N, self.LGs), device=dev),
                     offspring_loc=torch.zeros(N, dtype=torch.int64, device=dev), gen=torch.zeros((), dtype=torch.int64, device=dev), key=key)

    def init_tell(self, state, fitness):
        return state.update(fitness=fitness, inner_obj=fitness)

    def ask(self, state):
        key, per_key, sel_key, x_key, mut_key = rnd.split(state.key, 5)
        N, T = self.pop_size, self.T
        dev = state.population.device
        s = state.s.sum(1) + 1e-6
        d = s / s.sum() + 0.002
        d = d / d.sum()
        _, loc = self.selection(sel_key, state.inner_pop, 1.0 / d)
        B = state.B.gather(1, torch.argsort(rnd.uniform(per_key, (N, T)).to(dev), dim=1))
        parent = B[loc][:, :2]
        parents = torch.cat([state.inner_pop[parent[:, 0]], state.inner_pop[parent[:, 1]]], 0)
        off = self.mutation(mut_key, self.crossover(x_key, parents))
        return off, state.update(next_generation=off, offspring_loc=loc, key=key)

    def tell(self, state, fitness):
        N = self.pop_size
        gen = state.gen + 1
        P = state.B[state.offspring_loc]
        owner, inner_obj, _ = mo_ops.moead_scan(state.inner_obj, fitness, P, state.weight_vector,
                                                torch.zeros(self.n_objs, device=fitness.device), "weighted_sum", nr=self.T)
        inner_pop = torch.where((owner >= 0)[:, None], state.next_generation[owner.clamp(min=0)], state.inner_pop)
        merged_pop = torch.cat([state.population, state.next_generation], 0)
        merged_fit = torch.cat([state.fitness, fitness], 0)
        order = nsga2_select(merged_fit, N)
        survived_off = order >= N
        loc = state.offspring_loc[(order - N).clamp(min=0)]
        hist = torch.zeros(N, device=fitness.device).scatter_add_(0, loc, survived_off.to(torch.float32))
        col = (gen % self.LGs)
        onehot = torch.arange(self.LGs, device=fitness.device) == col
        s = torch.where((survived_off.any() & onehot)[None, :], hist[:, None], state.s)
        return state.update(population=merged_pop[order], fitness=merged_fit[order], inner_pop=inner_pop, inner_obj=inner_obj, s=s, gen=gen)
