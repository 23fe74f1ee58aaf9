"""Natural evolution strategies: exponential NES and separable NES
(reference ``es_variants/nes.py:20-209``).

XNES keeps ``A = σ·B`` with ``det B = 1``; the natural-gradient step on ``B`` uses the
matrix exponential (``torch.linalg.matrix_exp``).  The reference's SeparableNES calls
an undefined ``sort_key_valrows`` (``nes.py:188``) and cannot run; here it sorts the
population and its standard-normal samples by fitness, which is what that call meant.
"""
from __future__ import annotations

import math

import torch

from ....core import Algorithm, State
from ....ops import random as rnd
from ._common import sort_by_key


def _nes_weights(pop_size, device):
    w = math.log(pop_size / 2 + 1) - torch.log(torch.arange(1, pop_size + 1, dtype=torch.float32))
    w = torch.clamp(w, min=0)
    return (w / w.sum() - 1 / pop_size).to(device)


class XNES(Algorithm):
    def __init__(self, init_mean, init_covar, pop_size=None, recombination_weights=None, learning_rate_mean=None,
                 learning_rate_var=None, learning_rate_B=None, covar_as_cholesky=False):
        super().__init__()
        self.dim = init_mean.shape[0]
        self.init_mean = init_mean
        self.pop_size = 4 + math.floor(3 * math.log(self.dim)) if pop_size is None else pop_size
        assert self.pop_size > 0
        self.learning_rate_mean = 1 if learning_rate_mean is None else learning_rate_mean
        self.learning_rate_var = (9 + 3 * math.log(self.dim)) / 5 / math.pow(self.dim, 1.5) if learning_rate_var is None else learning_rate_var
        self.learning_rate_B = self.learning_rate_var if learning_rate_B is None else learning_rate_B
        assert self.learning_rate_mean > 0 and self.learning_rate_var > 0 and self.learning_rate_B > 0
        self.init_covar = init_covar if covar_as_cholesky else torch.linalg.cholesky(init_covar)
        w = _nes_weights(self.pop_size, init_mean.device) if recombination_weights is None else recombination_weights
        assert bool((w[1:] <= w[:-1]).all()), "recombination_weights must be in descending order"
        self.recombination_weights = w

    def setup(self, key):
        sigma = torch.pow(torch.prod(torch.diag(self.init_covar)), 1 / self.dim)
        B = self.init_covar / sigma
        return State(noise=torch.zeros((self.pop_size, self.dim), device=self.init_mean.device), mean=self.init_mean.clone(),
                     sigma=sigma, B=B, key=key)

    def ask(self, state):
        key, normal_key = rnd.split(state.key)
        noise = rnd.normal(normal_key, (self.pop_size, self.dim)).to(state.mean.device)
        return state.mean + state.sigma * (noise @ state.B.T), state.update(noise=noise, key=key)

    def tell(self, state, fitness):
        _, noise = sort_by_key(fitness, state.noise)
        w = self.recombination_weights
        I = torch.eye(self.dim, device=noise.device)
        grad_delta = (w[:, None] * noise).sum(0)
        grad_M = (w * noise.T) @ noise - w.sum() * I
        grad_sigma = torch.trace(grad_M) / self.dim
        grad_B = grad_M - grad_sigma * I
        mean = state.mean + self.learning_rate_mean * state.sigma * state.B @ grad_delta
        sigma = state.sigma * torch.exp(self.learning_rate_var / 2 * grad_sigma)
        B = state.B @ torch.linalg.matrix_exp(self.learning_rate_B / 2 * grad_B)
        return state.update(mean=mean, sigma=sigma, B=B)


class SeparableNES(Algorithm):
    def __init__(self, init_mean, init_std, pop_size=None, recombination_weights=None, learning_rate_mean=None,
                 learning_rate_var=None):
        super().__init__()
        self.dim = init_mean.shape[0]
        self.init_mean = init_mean
        assert init_std.shape == (self.dim,)
        self.init_std = init_std
        self.pop_size = 4 + math.floor(3 * math.log(self.dim)) if pop_size is None else pop_size
        self.learning_rate_mean = 1 if learning_rate_mean is None else learning_rate_mean
        self.learning_rate_var = (3 + math.log(self.dim)) / 5 / math.sqrt(self.dim) if learning_rate_var is None else learning_rate_var
        self.weight = _nes_weights(self.pop_size, init_mean.device) if recombination_weights is None else recombination_weights

    def _new_pop(self, key, mean, sigma):
        key, sample_key = rnd.split(key)
        z = rnd.normal(sample_key, (self.pop_size, self.dim)).to(mean.device)
        return mean + sigma * z, z, key

    def setup(self, key):
        pop, z, key = self._new_pop(key, self.init_mean, self.init_std)
        return State(population=pop, zero_mean_pop=z, mean=self.init_mean.clone(), sigma=self.init_std.clone(), key=key)

    def ask(self, state):
        return state.population, state

    def tell(self, state, fitness):
        _, z = sort_by_key(fitness, state.zero_mean_pop)
        w = self.weight[:, None]
        grad_mu = (w * z).sum(0)
        grad_sigma = (w * (z * z - 1)).sum(0)
        mean = state.mean + self.learning_rate_mean * state.sigma * grad_mu
        sigma = state.sigma * torch.exp(self.learning_rate_var / 2 * grad_sigma)
        pop, z, key = self._new_pop(state.key, mean, sigma)
        return state.update(population=pop, zero_mean_pop=z, mean=mean, sigma=sigma, key=key)
