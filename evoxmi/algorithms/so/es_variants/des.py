"""DES — discovered ES (Lange et al. 2023; reference ``es_variants/des.py:26-75``)."""
from __future__ import annotations

import torch

from ....core import Algorithm, State
from ....ops import random as rnd
from ....parallel.dim_sharded import ColumnSeparable


def get_des_weights(popsize: int, temperature: float = 12.5):
    ranks = torch.arange(popsize, dtype=torch.float32) / (popsize - 1) - 0.5
    return torch.softmax(-20 * torch.sigmoid(temperature * ranks), 0)


class DES(ColumnSeparable, Algorithm):
    # decision-axis state sharding (P2): centre, σ and the samples are column blocks
    column_separable = True
    dim_fields = ("sigma", "center", "x")

    def __init__(self, pop_size, center_init, temperature=12.5, sigma_init=0.1, mean_decay=0.0):
        super().__init__()
        self.num_dims = center_init.shape[0]
        self.dim = self.num_dims
        self.center_init = center_init
        self.popsize = pop_size
        self.sigma_init = sigma_init
        self.temperature = temperature
        self.lrate_sigma = 0.1
        self.lrate_mean = 1.0

    def setup(self, key):
        dev = self.center_init.device
        return State(key=key, sigma=self.sigma_init * torch.ones(self.num_dims, device=dev), center=self.center_init.clone(),
                     weights=get_des_weights(self.popsize, self.temperature).reshape(-1, 1).to(dev),
                     x=torch.zeros((self.popsize, self.num_dims), device=dev))

    def ask(self, state):
        key, _ = rnd.split(state.key)
        z = self.normal_cols(state.key, self.popsize, state.center.device)
        x = state.center + z * state.sigma[None, :]
        return x, state.update(key=key, x=x)

    def tell(self, state, fitness):
        x = state.x[torch.argsort(fitness, stable=True)]
        w = state.weights
        weighted_mean = (w * x).sum(0)
        weighted_sigma = torch.sqrt((w * (x - state.center) ** 2).sum(0) + 1e-6)
        center = state.center + self.lrate_mean * (weighted_mean - state.center)
        sigma = state.sigma + self.lrate_sigma * (weighted_sigma - state.sigma)
        return state.update(center=center, sigma=sigma)
