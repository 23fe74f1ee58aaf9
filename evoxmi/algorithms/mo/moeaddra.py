"""MOEA/D-DRA — dynamical resource allocation (Zhang et al. 2009; reference ``algorithms/mo/moeaddra.py:24-203``).

Utility-driven tournament picks the subproblems to work on (boundary subproblems
always), DE/rand/1 + polynomial mutation, and a *sequential* Tchebycheff
replacement with the ideal point updated per offspring and at most ``nr``
replacements each — run as one wave-level HIP kernel (``ops.mo.moead_scan``)
instead of N dependent steps; the utilities π are refreshed every 10 generations.
"""
from __future__ import annotations

import math

import torch

from ...core import State
from ...operators import crossover, selection
from ...operators.sampling import LatinHypercubeSampling
from ...ops import mo as mo_ops
from ...ops import random as rnd
from .common import MOAlgorithm, weights_and_neighbours


class MOEADDRA(MOAlgorithm):
    def __init__(self, lb, ub, n_objs, pop_size, mutation_op=None, crossover_op=None):
        super().__init__(lb, ub, n_objs, pop_size, mutation_op, crossover_op if crossover_op is not None else crossover.DifferentialEvolve())
        self.T = int(math.ceil(pop_size / 10))
        self.nr = int(math.ceil(pop_size / 100))
        self.i_size = int(math.floor(pop_size / 5))
        self.selection = selection.Tournament(n_round=pop_size)
        self.sample = LatinHypercubeSampling(pop_size, n_objs)

    def setup(self, key):
        key, k1, k2 = rnd.split(key, 3)
        pop = self._init_pop(k1)
        dev = pop.device
        w = self.sample(k2)[0].to(dev)
        N = self.pop_size
        return State(population=pop, fitness=torch.zeros((N, self.n_objs), device=dev), next_generation=pop, weight_vector=w,
                     B=weights_and_neighbours(w, self.T), Z=torch.zeros(self.n_objs, device=dev), pi=torch.ones(N, device=dev),
                     old_obj=torch.zeros(N, device=dev), choosed_p=torch.zeros((N, self.T), dtype=torch.int64, device=dev),
                     I_all=torch.zeros(N, dtype=torch.int64, device=dev), gen=torch.zeros((), dtype=torch.int64, device=dev), key=key)

    def init_tell(self, state, fitness):
        Z = fitness.min(0).values
        old_obj = (torch.abs(fitness - Z) * state.weight_vector).amax(1)
        return state.update(fitness=fitness, Z=Z, old_obj=old_obj)

    def ask(self, state):
        key, k1, k2, k3, sel_key, x_key, mut_key = rnd.split(state.key, 7)
        N, T = self.pop_size, self.T
        dev = state.population.device
        perm = torch.argsort(rnd.uniform(k1, (N, T)).to(dev), dim=1)
        parent = state.B.gather(1, perm)
        rand = rnd.uniform(k2, (N, 1)).to(dev)
        rand_perm = rnd.randint(k3, (N, T), 0, N).to(dev)
        _, sel_idx = self.selection(sel_key, state.population, -state.pi)
        w = state.weight_vector
        boundary_mask = (w < 1e-3).sum(1) == (self.n_objs - 1)
        # reference :103-106: boundary subproblems first (index 0 means "none"), tiled 5×
        bidx = torch.argsort((~boundary_mask).to(torch.int64), stable=True)
        bidx = torch.where(boundary_mask[bidx], bidx, torch.zeros_like(bidx))[: self.i_size]
        g_bound = bidx.repeat(5)
        g_bound = torch.cat([g_bound, torch.zeros(N - g_bound.shape[0], dtype=g_bound.dtype, device=dev)])[:N]
        I_all = torch.where(g_bound != 0, g_bound, sel_idx)
        choosed_p = torch.where(rand < 0.9, parent[I_all], rand_perm)
        pop = state.population
        off = self.crossover(x_key, pop[I_all], pop[choosed_p[:, 0]], pop[choosed_p[:, 1]])
        off = self.mutation(mut_key, off)
        return off, state.update(next_generation=off, choosed_p=choosed_p, key=key, I_all=I_all)

    def tell(self, state, fitness):
        gen = state.gen + 1
        owner, pop_obj, Z = mo_ops.moead_scan(state.fitness, fitness, state.choosed_p, state.weight_vector, state.Z,
                                              "tchebycheff", nr=self.nr, update_z=True)
        population = torch.where((owner >= 0)[:, None], state.next_generation[owner.clamp(min=0)], state.population)
        new_obj = (torch.abs(pop_obj - Z) * state.weight_vector).amax(1)
        delta = (state.old_obj - new_obj) / state.old_obj
        upd_pi = torch.where(delta < 0.001, state.pi * (0.95 + 0.05 * delta / 0.001), torch.ones_like(state.pi))
        refresh = (gen % 10) == 0
        return state.update(population=population, fitness=pop_obj, Z=Z, gen=gen, pi=torch.where(refresh, upd_pi, state.pi),
                            old_obj=torch.where(refresh, new_obj, state.old_obj))
