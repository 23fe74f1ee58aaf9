"""OpenES (Salimans et al. 2017; reference ``es_variants/open_es.py:19-82``).

Mirrored sampling ``ε, −ε``, gradient ``εᵀ f / (N σ)`` (one GEMV on the matrix
cores via hipBLAS), plain SGD step or an optimiser sub-module (``optimizer='adam'``).

SPMD protocol (north-star config 4, population sharded over the GPUs of a node):
``ask_sharded`` regenerates only this rank's rows of the (virtual, mirrored) noise
matrix from the Philox counters — row ``g`` is ``half[g]`` or ``−half[g − N/2]``
exactly as in ``ask`` — and ``tell_sharded`` all-reduces the rank's partial
gradient ``ε_localᵀ f_local`` (P floats) over RCCL; the centre/optimiser state
stays replicated and bit-identical on every rank.
"""
from __future__ import annotations

import torch

from ....core import Algorithm, State, use_state
from ....ops import random as rnd
from ._common import make_optimizer


class OpenES(Algorithm):
    rank_local_fields = ("population", "noise")

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

    # ------------------------------------------------------------------ SPMD protocol
    def _noise_rows(self, key, start: int, size: int, dev):
        d = self.dim
        if not self.mirrored_sampling:
            return rnd.normal(key, (size, d), offset=start * d).to(dev)
        h = self.pop_size // 2
        parts = []
        a0, a1 = start, min(start + size, h)
        if a1 > a0:
            parts.append(rnd.normal(key, (a1 - a0, d), offset=a0 * d).to(dev))
        b0, b1 = max(start, h) - h, start + size - h
        if b1 > b0:
            parts.append(-rnd.normal(key, (b1 - b0, d), offset=b0 * d).to(dev))
        return parts[0] if len(parts) == 1 else torch.cat(parts, 0)

    def ask_sharded(self, state, dist):
        start, size = dist.slice_of(self.pop_size)
        key, noise_key = rnd.split(state.key)
        noise = self._noise_rows(noise_key, start, size, state.center.device)
        population = state.center[None, :] + self.noise_stdev * noise
        return population, state.update(population=population, key=key, noise=noise)

    def tell_sharded(self, state, fitness, dist):
        start, size = dist.slice_of(self.pop_size)
        g = state.noise.T @ fitness[start : start + size].to(state.noise.dtype)
        dist.all_reduce_(g)
        grad = g / self.pop_size / self.noise_stdev
        if self.optimizer is None:
            center = state.center - self.learning_rate * grad
        else:
            updates, state = use_state(self.optimizer.update)(state, grad, state.center)
            center = state.center + updates
        return state.update(center=center)
