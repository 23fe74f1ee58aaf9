"""Noise-reuse ES (Li et al. 2023; reference ``es_variants/noise_reuse_es.py:19-105``).

One antithetic perturbation is reused for all K-step truncations of an unroll of length T.
"""
from __future__ import annotations

import torch

from ....core import Algorithm, State, use_state
from ....ops import random as rnd
from ._common import make_optimizer


class NoiseReuseES(Algorithm):
    def __init__(self, pop_size, center_init, optimizer="adam", lr=0.05, sigma=0.03, T=100, K=10, lrate_decay=1.0,
                 lrate_limit=0.001, sigma_decay=1.0, sigma_limit=0.01, sigma_lrate=0.2, init_min=0.0, init_max=0.0,
                 clip_min=None, clip_max=None):
        super().__init__()
        if optimizer not in ("adam", "sgd"):
            raise NotImplementedError
        self.num_dims = center_init.shape[0]
        self.center_init = center_init
        self.popsize = pop_size
        self.lr, self.sigma, self.T, self.K = lr, sigma, T, K
        self.sigma_decay, self.sigma_limit = sigma_decay, sigma_limit
        self.optimizer = make_optimizer(optimizer, lr, center_init)

    def setup(self, key):
        dev = self.center_init.device
        z = torch.zeros((self.popsize, self.num_dims), device=dev)
        return State(key=key, unroll_pert=z, center=self.center_init.clone(), population=z.clone(),
                     inner_step_counter=torch.zeros((), dtype=torch.int64, device=dev), sigma=torch.tensor(float(self.sigma), device=dev))

    def ask(self, state):
        key, _ = rnd.split(state.key)
        pos = rnd.normal(state.key, (self.popsize // 2, self.num_dims)).to(state.center.device) * state.sigma
        perts = torch.cat([pos, -pos], 0)
        unroll = torch.where(state.inner_step_counter == 0, perts, state.unroll_pert)
        x = state.center + unroll
        return x, state.update(key=key, unroll_pert=unroll, population=x)

    def tell(self, state, fitness):
        theta_grad = (state.unroll_pert * fitness[:, None] / (state.sigma**2)).mean(0)
        updates, state = use_state(self.optimizer.update)(state, theta_grad, state.center)
        counter = state.inner_step_counter + self.K
        reset = counter >= self.T
        return state.update(center=state.center + updates, inner_step_counter=torch.where(reset, torch.zeros_like(counter), counter),
                            sigma=torch.clamp(self.sigma_decay * state.sigma, min=self.sigma_limit))


Noise_reuse_es = NoiseReuseES  # reference class name
