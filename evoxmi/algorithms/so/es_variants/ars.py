"""ARS — augmented random search (Mania et al. 2018; reference ``es_variants/ars.py:19-82``)."""
from __future__ import annotations

import torch

from ....core import Algorithm, State, use_state
from ....ops import random as rnd
from ....parallel.dim_sharded import ColumnSeparable
from ._common import make_optimizer


class ARS(ColumnSeparable, Algorithm):
    # decision-axis state sharding (P2): centre, population, noise and Adam's moments are column
    # blocks; elite choice and the fitness scale come from the replicated fitness
    column_separable = True
    dim_fields = ("center", "population", "noise")
    dim_child_fields = {"optimizer": ("opt_state",)}

    def __init__(self, pop_size, center_init, elite_ratio=0.1, optimizer="adam", lr=0.05, sigma=0.03):
        super().__init__()
        assert not pop_size & 1
        assert 0 <= elite_ratio <= 1
        if optimizer != "adam":
            raise NotImplementedError
        self.dim = center_init.shape[0]
        self.center_init = center_init
        self.pop_size = pop_size
        self.lr, self.sigma, self.elite_ratio = lr, sigma, elite_ratio
        self.elite_pop_size = max(1, int(self.pop_size / 2 * self.elite_ratio))
        self.optimizer = make_optimizer(optimizer, lr, center_init)

    def setup(self, key):
        dev = self.center_init.device
        z = torch.zeros((self.pop_size, self.dim), device=dev)
        return State(key=key, center=self.center_init.clone(), population=z, noise=z.clone())

    def ask(self, state):
        key, _ = rnd.split(state.key)
        z_plus = self.normal_cols(state.key, self.pop_size // 2, state.center.device)
        z = torch.cat([z_plus, -z_plus])
        x = state.center + self.sigma * z
        return x, state.update(key=key, population=x, noise=z)

    def tell(self, state, fitness):
        h = self.pop_size // 2
        noise_1, fit_1, fit_2 = state.noise[:h], fitness[:h], fitness[h:]
        elite = torch.argsort(torch.minimum(fit_1, fit_2), stable=True)[: self.elite_pop_size]
        fitness_elite = torch.cat([fit_1[elite], fit_2[elite]])
        sigma_fitness = fitness_elite.std(unbiased=False) + 1e-5
        theta_grad = (noise_1[elite].T @ (fit_1[elite] - fit_2[elite])) / (self.elite_pop_size * sigma_fitness)
        updates, state = use_state(self.optimizer.update)(state, theta_grad, state.center)
        return state.update(center=state.center + updates)
