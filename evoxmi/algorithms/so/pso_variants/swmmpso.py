"""Small-world-network PSO (reference ``pso_variants/swmmpso.py:24-161``): K-nearest
"circles" neighbourhood with random shortcut rewiring, neighbourhood-best PSO with
Clerc's constriction."""
from __future__ import annotations

import torch

from ....core import Algorithm, State
from ....ops import random as rnd
from .topology_utils import build_adjacancy_list_from_matrix, get_circles_neighbour, get_neighbour_best_fitness
from .utils import init_swarm


class SwmmPSO(Algorithm):
    def __init__(self, lb, ub, pop_size, max_phi_1=2.05, max_phi_2=2.05, max_phi=4.1, mean=None, stdev=None, topology="Circles", shortcut=0):
        super().__init__()
        self.dim = lb.shape[0]
        self.lb, self.ub, self.pop_size = lb, ub, pop_size
        self.max_phi_1, self.max_phi_2, self.max_phi = max_phi_1, max_phi_2, max_phi
        self.mean, self.stdev, self.topology, self.shortcut = mean, stdev, topology, shortcut

    def setup(self, key):
        state_key, kp, kv, k_adj = rnd.split(key, 4)
        pop, vel = init_swarm(kp, kv, self.pop_size, self.lb, self.ub, self.mean, self.stdev)
        phi_v = self.max_phi if self.max_phi > 0 else self.max_phi_1 + self.max_phi_2
        phi = torch.full((self.pop_size, 1), float(phi_v), device=pop.device)
        chi = 2 / (phi - 2 + torch.sqrt(torch.abs(phi * (phi - 4))))
        if self.topology != "Circles":
            raise NotImplementedError(self.topology)
        adj = get_circles_neighbour(k_adj, pop, K=2, shortcut=self.shortcut)
        lst, _ = build_adjacancy_list_from_matrix(adj)
        inf = torch.full((self.pop_size,), float("inf"), device=pop.device)
        return State(population=pop, velocity=vel, local_best_location=pop, local_best_fitness=inf, neighbour_best_location=pop,
                     neighbour_best_fitness=inf.clone(), adjacancy_matrix=adj, nb_list=lst, key=state_key, chi=chi, phi=phi)

    def ask(self, state):
        return state.population, state

    def tell(self, state, fitness):
        key, k1, k2, _ = rnd.split(state.key, 4)
        dev = fitness.device
        phi1 = rnd.uniform(k1, (self.pop_size, self.dim)).to(dev) * self.max_phi_1
        phi2 = rnd.uniform(k2, (self.pop_size, self.dim)).to(dev) * self.max_phi_2
        better = state.local_best_fitness > fitness
        lbl = torch.where(better[:, None], state.population, state.local_best_location)
        lbf = torch.minimum(state.local_best_fitness, fitness)
        nbf, nbi = get_neighbour_best_fitness(lbf, state.nb_list)
        nbl = lbl[nbi]
        velocity = state.chi * (state.velocity + phi1 * (lbl - state.population) + phi2 * (nbl - state.population))
        population = torch.clamp(state.population + velocity, self.lb, self.ub)
        return state.update(population=population, velocity=velocity, local_best_location=lbl, local_best_fitness=lbf,
                            neighbour_best_location=nbl, neighbour_best_fitness=nbf, key=key)
