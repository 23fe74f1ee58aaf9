"""Fully-informed PSO (Mendes et al. 2004; reference ``pso_variants/fips.py:20-199``).

Every particle moves towards the φ-weighted average of its neighbours' personal
bests (Square/von Neumann or All topology; constant, pbest-fitness or distance
weights) with Clerc's constriction χ.  The reference draws an (N, N, d) random
tensor per step (O(N² d) memory); the same estimator is computed here as a batched
weighted average over the padded neighbour list, (N, K, d) with K = max degree.
"""
from __future__ import annotations

import math

import torch

from ....core import Algorithm, State
from ....ops import random as rnd
from .topology_utils import build_adjacancy_list_from_matrix, get_full_neighbour, get_square_neighbour
from .utils import get_distance_matrix, init_swarm


class FIPS(Algorithm):
    def __init__(self, lb, ub, pop_size, max_phi=4.1, mean=None, stdev=None, topology="Square", weight_type="Distance", shortcut=0):
        super().__init__()
        self.dim = lb.shape[0]
        self.lb, self.ub, self.pop_size = lb, ub, pop_size
        self.max_phi, self.mean, self.stdev = max_phi, mean, stdev
        self.topology, self.weight_type, self.shortcut = topology, weight_type, shortcut

    def setup(self, key):
        state_key, kp, kv = rnd.split(key, 3)
        pop, vel = init_swarm(kp, kv, self.pop_size, self.lb, self.ub, self.mean, self.stdev)
        if self.topology in ("Square", "USquare"):
            adj = get_square_neighbour(pop)
        elif self.topology in ("All", "UAll"):
            adj = get_full_neighbour(pop)
        else:
            raise NotImplementedError(self.topology)
        lst, mask = build_adjacancy_list_from_matrix(adj)
        K = int(mask.sum(1).max())
        phi = torch.full((self.pop_size, 1), float(self.max_phi), device=pop.device)
        chi = 2 / (phi - 2 + torch.sqrt(torch.abs(phi * (phi - 4))))
        inf = torch.full((self.pop_size,), float("inf"), device=pop.device)
        return State(population=pop, velocity=vel, local_best_location=pop, local_best_fitness=inf, neighbour_best_location=pop,
                     neighbour_best_fitness=inf.clone(), adjacancy_matrix=adj, nb_list=lst[:, :K].contiguous(),
                     nb_mask=mask[:, :K].to(torch.float32).contiguous(), key=state_key, chi=chi, phi=phi)

    def ask(self, state):
        return state.population, state

    def tell(self, state, fitness):
        key, k1 = rnd.split(state.key)
        better = state.local_best_fitness > fitness
        lbl = torch.where(better[:, None], state.population, state.local_best_location)
        lbf = torch.minimum(state.local_best_fitness, fitness)
        lst, mask = state.nb_list, state.nb_mask
        if self.weight_type == "Constant":
            w = torch.ones_like(mask)
        elif self.weight_type == "Pbest":
            w = 1 / lbf[lst]
        else:
            w = get_distance_matrix(lbl).gather(1, lst)
        N, K = lst.shape
        phik = rnd.uniform(k1, (N, K, self.dim)).to(fitness.device) * mask[:, :, None] * self.max_phi
        wp = w[:, :, None] * phik
        pm = (lbl[lst] * wp).sum(1) / wp.sum(1)
        velocity = state.chi * (state.velocity + state.phi * (pm - state.population))
        population = torch.clamp(state.population + velocity, self.lb, self.ub)
        return state.update(population=population, velocity=velocity, local_best_location=lbl, local_best_fitness=lbf, key=key)
