"""ESMC — ES with a mirrored baseline member (Merchant et al. 2021; reference ``es_variants/esmc.py:18-93``)."""
from __future__ import annotations

import torch

from ....core import Algorithm, State, use_state
from ....ops import random as rnd
from ._common import make_optimizer


class ESMC(Algorithm):
    def __init__(self, pop_size, center_init, optimizer="adam", lrate_decay=1.0, lrate_limit=0.001, sigma_decay=1.0,
                 sigma_limit=0.01, lr=0.05, sigma=0.03, init_min=0.0, init_max=0.0, clip_min=None, clip_max=None):
        super().__init__()
        assert pop_size & 1
        if optimizer not in ("adam", "sgd"):
            raise NotImplementedError
        self.num_dims = center_init.shape[0]
        self.center_init = center_init
        self.popsize = pop_size
        self.lr, self.sigma = lr, sigma
        self.sigma_decay, self.sigma_limit = sigma_decay, sigma_limit
        self.lrate_decay, self.lrate_limit = lrate_decay, lrate_limit
        self.optimizer = make_optimizer(optimizer, lr, center_init)

    def setup(self, key):
        dev = self.center_init.device
        return State(key=key, center=self.center_init.clone(), sigma=torch.ones(self.num_dims, device=dev) * self.sigma,
                     x=torch.zeros((self.popsize, self.num_dims), device=dev))

    def ask(self, state):
        key, _ = rnd.split(state.key)
        h = self.popsize // 2
        z_plus = rnd.normal(state.key, (h, self.num_dims)).to(state.center.device)
        z = torch.cat([torch.zeros_like(z_plus[:1]), z_plus, -z_plus])
        x = state.center + z * state.sigma[None, :]
        return x, state.update(key=key, x=x)

    def tell(self, state, fitness):
        noise = ((state.x - state.center) / state.sigma)[1:]
        base = fitness[0]
        fit = fitness[1:]
        h = (self.popsize - 1) // 2
        fit_diff = torch.minimum(fit[:h], base) - torch.minimum(fit[h:], base)
        theta_grad = (noise[:h].T @ fit_diff) / h
        updates, state = use_state(self.optimizer.update)(state, theta_grad, state.center)
        sigma = torch.clamp(state.sigma * self.sigma_decay, min=self.sigma_limit)
        return state.update(center=state.center + updates, sigma=sigma)
