"""SNES — separable NES, evosax flavour (reference ``es_variants/snes.py:34-86``)."""
from __future__ import annotations

import math

import torch

from ....core import Algorithm, State
from ....parallel.dim_sharded import ColumnSeparable
from ....ops import random as rnd


def get_recombination_weights(popsize: int, use_baseline: bool = True):
    w = torch.clamp(math.log(popsize / 2 + 1) - torch.log(torch.arange(1, popsize + 1, dtype=torch.float32)), min=0)
    return w / w.sum() - use_baseline * (1 / popsize)


def get_temp_weights(popsize: int, temperature: float):
    ranks = torch.arange(popsize, dtype=torch.float32) / (popsize - 1) - 0.5
    return torch.softmax(-temperature * ranks, 0)


class SNES(ColumnSeparable, Algorithm):
    # decision-axis state sharding (P2): centre, σ, noise and population are column blocks;
    # each rank draws only its columns of the Philox noise (normal_cols), the update weights
    # come from the replicated fitness ranks
    column_separable = True
    dim_fields = ("sigma", "center", "noise", "population")

    def __init__(self, pop_size, center_init, sigma=1.0, lrate_mean=1.0, temperature=0.0, init_min=0.0, init_max=0.0):
        super().__init__()
        self.num_dims = center_init.shape[0]
        self.dim = self.num_dims
        self.center_init = center_init
        self.popsize = pop_size
        self.sigma = sigma
        self.lrate_mean = lrate_mean
        self.lrate_sigma = (3 + math.log(self.num_dims)) / (5 * math.sqrt(self.num_dims))
        self.temperature = temperature
        self.init_min, self.init_max = init_min, init_max

    def setup(self, key):
        w = get_temp_weights(self.popsize, self.temperature) if self.temperature > 0.0 else get_recombination_weights(self.popsize)
        dev = self.center_init.device
        return State(key=key, sigma=self.sigma * torch.ones(self.num_dims, device=dev), center=self.center_init.clone(),
                     weights=w.reshape(-1, 1).to(dev), noise=torch.zeros((self.popsize, self.num_dims), device=dev),
                     population=torch.zeros((self.popsize, self.num_dims), device=dev))

    def ask(self, state):
        key, _ = rnd.split(state.key)
        noise = self.normal_cols(key, self.popsize, state.center.device)
        x = state.center + noise * state.sigma[None, :]
        return x, state.update(key=key, noise=noise, population=x)

    def tell(self, state, fitness):
        s = state.noise[torch.argsort(fitness, stable=True)]
        grad_mean = (state.weights * s).sum(0)
        grad_sigma = (state.weights * (s * s - 1)).sum(0)
        center = state.center + self.lrate_mean * state.sigma * grad_mean
        sigma = state.sigma * torch.exp(self.lrate_sigma / 2 * grad_sigma)
        return state.update(center=center, sigma=sigma)
