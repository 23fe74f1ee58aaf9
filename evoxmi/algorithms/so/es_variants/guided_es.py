"""Guided ES (Maheswaranathan et al. 2019; reference ``es_variants/guided_es.py:18-109``).

Antithetic samples from ``σ√(α/d)·ε_full + σ√((1−α)/k)·Q ε_sub`` where Q is an
orthonormal basis (QR, ``torch.linalg.qr``) of the k most recent surrogate gradients.
"""
from __future__ import annotations

import math

import torch

from ....core import Algorithm, State, use_state
from ....ops import random as rnd
from ._common import make_optimizer


class GuidedES(Algorithm):
    def __init__(self, pop_size, center_init, subspace_dims=1, optimizer="sgd", sigma_init=0.03, lrate_init=60,
                 lrate_decay=1.0, lrate_limit=0.001, sigma_decay=1.0, sigma_limit=0.01, mean_decay=0.0):
        super().__init__()
        assert pop_size % 2 == 0
        if optimizer not in ("adam", "sgd"):
            raise NotImplementedError
        self.num_dims = center_init.shape[0]
        self.center_init = center_init
        self.popsize = pop_size
        self.lr, self.sigma = lrate_init, sigma_init
        self.subspace_dims = subspace_dims
        self.sigma_decay, self.sigma_limit = sigma_decay, sigma_limit
        self.alpha, self.beta = 0.5, 1.0
        self.optimizer = make_optimizer(optimizer, lrate_init, center_init)

    def setup(self, key):
        dev = self.center_init.device
        return State(key=key, center=self.center_init.clone(), sigma=torch.tensor(float(self.sigma), device=dev),
                     grad_subspace=rnd.normal(key, (self.subspace_dims, self.num_dims)).to(dev),
                     z=torch.zeros((self.popsize, self.num_dims), device=dev))

    def ask(self, state):
        key, _ = rnd.split(state.key)
        a = state.sigma * math.sqrt(self.alpha / self.num_dims)
        c = state.sigma * math.sqrt((1.0 - self.alpha) / self.subspace_dims)
        key_full, key_sub = rnd.split(state.key, 2)
        dev = state.center.device
        h = self.popsize // 2
        eps_full = rnd.normal(key_full, (self.num_dims, h)).to(dev)
        eps_sub = rnd.normal(key_sub, (self.subspace_dims, h)).to(dev)
        z_plus = (a * eps_full + c * _proj(state.grad_subspace, eps_sub)).T
        z = torch.cat([z_plus, -z_plus])
        return state.center + z, state.update(key=key, z=z)

    def tell(self, state, fitness):
        h = self.popsize // 2
        noise = state.z / state.sigma
        theta_grad = (self.beta / self.popsize) * (noise[:h].T @ (fitness[:h] - fitness[h:]))
        grad_subspace = torch.cat([state.grad_subspace[1:], theta_grad[None]], 0)
        state = state.update(grad_subspace=grad_subspace)
        updates, state = use_state(self.optimizer.update)(state, theta_grad, state.center)
        sigma = torch.clamp(self.sigma_decay * state.sigma, min=self.sigma_limit)
        return state.update(center=state.center + updates, sigma=sigma)


def _proj(G, eps_sub):
    """Subspace term for the usual k < d case.

    The reference computes ``jnp.dot(Q, eps_subspace)`` with Q from ``qr`` of the
    (k, d) gradient matrix, i.e. a (k, k) factor, and the product only type-checks
    when k = d.  The method (Maheswaranathan et al.) samples in the span of the
    surrogate gradients: U ε_sub with U the (d, k) orthonormal basis of Gᵀ.
    """
    U, _ = torch.linalg.qr(G.T)  # (d, k)
    return U @ eps_sub
