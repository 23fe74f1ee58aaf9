"""OpenES (Salimans et al. 2017; reference ``es_variants/open_es.py:19-82``).

Mirrored sampling ``ε, −ε``, gradient ``εᵀ f / (N σ)`` (one GEMV on the matrix
cores via hipBLAS), plain SGD step or an optimiser sub-module (``optimizer='adam'``).
"""
from __future__ import annotations

import torch

from ....core import Algorithm, State, use_state
from ....ops import random as rnd
from ._common import make_optimizer


class OpenES(Algorithm):
    def __init__(self, center_init, pop_size, learning_rate, noise_stdev, optimizer=None, mirrored_sampling=True):
        super().__init__()
        assert noise_stdev > 0 and learning_rate > 0 and pop_size > 0
        if mirrored_sampling:
            assert pop_size % 2 == 0, "When mirrored_sampling is True, pop_size must be a multiple of 2."
        self.dim = center_init.shape[0]
        self.center_init = center_init
        self.pop_size = pop_size
        self.learning_rate = learning_rate
        self.noise_stdev = noise_stdev
        self.mirrored_sampling = mirrored_sampling
        self.optimizer = make_optimizer(optimizer, learning_rate, center_init) if optimizer == "adam" else None

    def setup(self, key):
        pop = self.center_init.expand(self.pop_size, -1).clone()
        return State(population=pop, center=self.center_init.clone(), noise=pop.clone(), key=key)

    def ask(self, state):
        key, noise_key = rnd.split(state.key)
        dev = state.center.device
        if self.mirrored_sampling:
            half = rnd.normal(noise_key, (self.pop_size // 2, self.dim)).to(dev)
            noise = torch.cat([half, -half], 0)
        else:
            noise = rnd.normal(noise_key, (self.pop_size, self.dim)).to(dev)
        population = state.center[None, :] + self.noise_stdev * noise
        return population, state.update(population=population, key=key, noise=noise)

    def tell(self, state, fitness):
        grad = (state.noise.T @ fitness) / self.pop_size / self.noise_stdev
        if self.optimizer is None:
            center = state.center - self.learning_rate * grad
        else:
            updates, state = use_state(self.optimizer.update)(state, grad, state.center)
            center = state.center + updates
        return state.update(center=center)
