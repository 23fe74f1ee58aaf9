"""ASEBO — adaptive ES with active subspaces (Choromanski et al. 2019; reference ``es_variants/asebo.py:20-135``).

The gradient subspace is re-estimated with an SVD of the recent gradient history
(sign-fixed as sklearn's ``svd_flip``), samples come from a Cholesky factor of the
blended isotropic/subspace covariance and are normalised to unit length.
The reference computes the shifted gradient history in ``tell`` but never stores it
(``asebo.py:118-121``), so its subspace stays empty; here it is kept in the state.
"""
from __future__ import annotations

import torch

from ....core import Algorithm, State, use_state
from ....ops import random as rnd
from ._common import make_optimizer


class ASEBO(Algorithm):
    def __init__(self, pop_size, center_init, optimizer="adam", lr=0.05, lr_decay=1.0, lr_limit=0.001, sigma=0.03,
                 sigma_decay=1.0, sigma_limit=0.01, mean_decay=0.0, subspace_dims=50):
        super().__init__()
        assert not pop_size & 1
        if optimizer != "adam":
            raise NotImplementedError
        self.optimizer = make_optimizer(optimizer, lr, center_init)
        self.dim = center_init.shape[0]
        self.center_init = center_init
        self.pop_size = pop_size
        self.lr, self.sigma = lr, sigma
        self.sigma_decay, self.sigma_limit = sigma_decay, sigma_limit
        self.subspace_dims = subspace_dims

    def setup(self, key):
        dev = self.center_init.device
        d = self.dim
        return State(key=key, center=self.center_init.clone(), grad_subspace=torch.zeros((self.subspace_dims, d), device=dev),
                     gen_counter=torch.zeros((), dtype=torch.int64, device=dev), sigma=torch.tensor(float(self.sigma), device=dev),
                     alpha=torch.tensor(0.1, device=dev), population=torch.zeros((self.pop_size, d), device=dev),
                     noise=torch.zeros((self.pop_size, d), device=dev), UUT=torch.zeros((d, d), device=dev),
                     UUT_ort=torch.zeros((d, d), device=dev))

    def ask(self, state):
        key, rng = rnd.split(state.key)
        X = state.grad_subspace - state.grad_subspace.mean(0)
        U, S, Vt = torch.linalg.svd(X, full_matrices=False)
        # svd_flip: make the largest-|.| entry of each column of U positive
        cols = torch.arange(U.shape[1], device=U.device)
        signs = torch.sign(U[torch.argmax(U.abs(), 0), cols])
        Vt = Vt * signs[:, None]
        h = self.pop_size // 2
        Us = Vt[:h]
        UUT = Us.T @ Us
        U_ort = Vt[h:]
        UUT_ort = U_ort.T @ U_ort
        ready = state.gen_counter > self.subspace_dims
        UUT = torch.where(ready, UUT, torch.zeros_like(UUT))
        eye = torch.eye(self.dim, device=X.device)
        cov = state.sigma * (state.alpha / self.dim) * eye + ((1 - state.alpha) / h) * UUT
        chol = torch.linalg.cholesky(cov)
        noise = rnd.normal(rng, (self.dim, h)).to(X.device)
        z_plus = (chol @ noise).T
        z_plus = z_plus / torch.linalg.norm(z_plus, dim=-1, keepdim=True)
        z = torch.cat([z_plus, -z_plus])
        x = state.center + z
        return x, state.update(key=key, population=x, noise=z, UUT=UUT, UUT_ort=UUT_ort, gen_counter=state.gen_counter + 1)

    def tell(self, state, fitness):
        h = self.pop_size // 2
        noise = (state.population - state.center) / state.sigma
        theta_grad = 0.5 * (noise[:h].T @ (fitness[:h] - fitness[h:]))
        alpha = torch.linalg.norm(theta_grad @ state.UUT_ort) / torch.linalg.norm(theta_grad @ state.UUT)
        alpha = torch.where(state.gen_counter > self.subspace_dims, alpha, torch.ones_like(alpha))
        # keep the isotropic share positive so the sampling covariance stays PD (0/0 → NaN
        # and α = 0 occur once the subspace spans the gradient history)
        alpha = torch.nan_to_num(alpha, nan=1.0).clamp(1e-3, 1.0)
        grad_subspace = torch.cat([state.grad_subspace[1:], theta_grad[None]], 0)
        theta_grad = theta_grad / (torch.linalg.norm(theta_grad) / self.dim + 1e-8)
        updates, state = use_state(self.optimizer.update)(state, theta_grad, state.center)
        sigma = torch.clamp(state.sigma * self.sigma_decay, min=self.sigma_limit)
        return state.update(center=state.center + updates, sigma=sigma, alpha=alpha, grad_subspace=grad_subspace)
