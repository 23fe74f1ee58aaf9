"""Persistent ES for unrolled computation graphs (Vicol et al. 2021; reference ``es_variants/persistent_es.py:19-118``).

Perturbations are accumulated over the K-step truncations of an inner problem of
length T and reset when it completes.
"""
from __future__ import annotations

import torch

from ....core import Algorithm, State, use_state
from ....ops import random as rnd
from ._common import make_optimizer


class PersistentES(Algorithm):
    def __init__(self, pop_size, center_init, optimizer="adam", lr=0.05, sigma=0.03, T=100, K=10, lrate_decay=1.0,
                 lrate_limit=0.001, sigma_decay=1.0, sigma_limit=0.01, sigma_lrate=0.2, sigma_max_change=0.2, init_min=0.0,
                 init_max=0.0, clip_min=None, clip_max=None):
        super().__init__()
        assert pop_size % 2 == 0
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
        return State(key=key, center=self.center_init.clone(), inner_step_counter=torch.zeros((), dtype=torch.int64, device=dev),
                     sigma=torch.tensor(float(self.sigma), device=dev), pert_accum=z, population=z.clone())

    def ask(self, state):
        key, _ = rnd.split(state.key)
        pos = rnd.normal(state.key, (self.popsize // 2, self.num_dims)).to(state.center.device) * self.sigma
        perts = torch.cat([pos, -pos], 0)
        pert_accum = state.pert_accum + perts
        x = state.center + perts
        return x, state.update(key=key, pert_accum=pert_accum, population=x)

    def tell(self, state, fitness):
        theta_grad = (state.pert_accum * fitness[:, None] / (self.sigma**2)).mean(0)
        updates, state = use_state(self.optimizer.update)(state, theta_grad, state.center)
        counter = state.inner_step_counter + self.K
        reset = counter >= self.T
        return state.update(center=state.center + updates, sigma=torch.clamp(self.sigma_decay * state.sigma, min=self.sigma_limit),
                            pert_accum=torch.where(reset, torch.zeros_like(state.pert_accum), state.pert_accum),
                            inner_step_counter=torch.where(reset, torch.zeros_like(counter), counter))
