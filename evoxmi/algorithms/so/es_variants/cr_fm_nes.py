"""CR-FM-NES — cost-reduced fast-moving NES (Nomura & Ono 2022; reference ``es_variants/cr_fm_nes.py:44-222``).

Covariance ``σ² D (I + v vᵀ) D`` (diagonal + rank-one), updated through the
closed-form natural-gradient expressions of the paper; all operations are O(N·d).
"""
from __future__ import annotations

import math

import torch

from ....core import Algorithm, State
from ....ops import random as rnd


def get_recombination_weights(popsize: int):
    w_hat = math.log(popsize / 2 + 1) - torch.log(torch.arange(1, popsize + 1, dtype=torch.float32))
    w_hat = w_hat * (w_hat >= 0)
    w = w_hat / w_hat.sum() - 1.0 / popsize
    return w_hat.reshape(-1, 1), w.reshape(-1, 1)


def get_h_inv(dim: int):
    dim = min(dim, 2000)
    f = lambda a: ((1.0 + a * a) * math.exp(a * a / 2.0) / 0.24) - 10.0 - dim
    fp = lambda a: (1.0 / 0.24) * a * math.exp(a * a / 2.0) * (3.0 + a * a)
    h = 1.0
    while abs(f(h)) > 1e-10:
        h = h - 0.5 * (f(h) / fp(h))
    return h


class CR_FM_NES(Algorithm):
    def __init__(self, pop_size, center_init, sigma=0.03):
        super().__init__()
        assert pop_size % 2 == 0, "Population size must be even"
        d = center_init.shape[0]
        self.num_dims, self.center_init, self.popsize, self.sigma = d, center_init, pop_size, sigma
        w_hat, w = get_recombination_weights(pop_size)
        mueff = float(1 / ((w + 1 / pop_size).T @ (w + 1 / pop_size)))
        self.mu_eff = mueff
        self.c_s = (mueff + 2.0) / (d + mueff + 5.0)
        self.c_c = (4.0 + mueff / d) / (d + 4.0 + 2.0 * mueff / d)
        c1_cma = 2.0 / ((d + 1.3) ** 2 + mueff)
        self.chi_N = math.sqrt(d) * (1.0 - 1.0 / (4.0 * d) + 1.0 / (21.0 * d * d))
        self.h_inv = get_h_inv(d)
        self.alpha_dist = self.h_inv * min(1.0, math.sqrt(pop_size / d))
        self.lrate_move_sigma = 1.0
        self.lrate_stag_sigma = math.tanh((0.024 * pop_size + 0.7 * d + 20.0) / (d + 12.0))
        self.lrate_conv_sigma = 2.0 * math.tanh((0.025 * pop_size + 0.75 * d + 10.0) / (d + 4.0))
        self.c1 = c1_cma * (d - 5) / 6
        self.lrate_B = math.tanh((min(0.02 * pop_size, 3 * math.log(d)) + 5) / (0.23 * d + 25))
        self.lrate_mean = 1.0

    def setup(self, key):
        rng_init, rng_v = rnd.split(key)
        w_hat, w = get_recombination_weights(self.popsize)
        d, dev = self.num_dims, self.center_init.device
        return State(key=key, sigma=torch.tensor(float(self.sigma), device=dev), center=self.center_init.clone(),
                     v=rnd.normal(rng_v, (d, 1)).to(dev) / math.sqrt(d), D=torch.ones((d, 1), device=dev),
                     p_sigma=torch.zeros((d, 1), device=dev), p_c=torch.zeros((d, 1), device=dev),
                     z=torch.zeros((d, self.popsize), device=dev), y=torch.zeros((d, self.popsize), device=dev),
                     x=torch.zeros((self.popsize, d), device=dev), w_rank_hat=w_hat.to(dev), w_rank=w.to(dev))

    def ask(self, state):
        key, _ = rnd.split(state.key)
        z_plus = rnd.normal(state.key, (self.popsize // 2, self.num_dims)).to(state.center.device)
        z = torch.cat([z_plus, -z_plus]).T
        normv = torch.linalg.norm(state.v)
        vbar = state.v / normv
        y = z + (torch.sqrt(1 + normv**2) - 1) * vbar @ (vbar.T @ z)
        x = (state.center[:, None] + state.sigma * y * state.D).T
        return x, state.update(z=z, y=y, key=key, x=x)

    def tell(self, state, fitness):
        d, n = self.num_dims, self.popsize
        ranks = torch.argsort(fitness, stable=True)
        z, y, x = state.z[:, ranks], state.y[:, ranks], state.x.T[:, ranks]
        p_sigma = (1 - self.c_s) * state.p_sigma + math.sqrt(self.c_s * (2.0 - self.c_s) * self.mu_eff) * (z @ state.w_rank)
        p_sigma_norm = torch.linalg.norm(p_sigma)
        w_tmp = state.w_rank_hat * torch.exp(self.alpha_dist * torch.linalg.norm(z, dim=0)).reshape(-1, 1)
        weights_dist = w_tmp / w_tmp.sum() - 1.0 / n
        cond = p_sigma_norm >= self.chi_N
        weights = torch.where(cond, weights_dist, state.w_rank)
        zero = p_sigma_norm * 0  # device scalars without host→device copies (graph-capturable)
        lrate_sigma = torch.where(cond, zero + self.lrate_move_sigma, zero + self.lrate_stag_sigma)
        lrate_sigma = torch.where(p_sigma_norm >= 0.1 * self.chi_N, lrate_sigma, zero + self.lrate_conv_sigma)
        wxm = (x - state.center[:, None]) @ weights
        p_c = (1.0 - self.c_c) * state.p_c + math.sqrt(self.c_c * (2.0 - self.c_c) * self.mu_eff) * wxm / state.sigma
        center = state.center + self.lrate_mean * wxm.squeeze(1)
        normv = torch.linalg.norm(state.v)
        vbar = state.v / normv
        normv2 = normv**2
        normv4 = normv2**2
        exY = torch.cat([y, p_c / state.D], 1)
        yy = exY * exY
        ip_yvbar = vbar.T @ exY
        yvbar = exY * vbar
        gammav = 1.0 + normv2
        vbarbar = vbar * vbar
        alphavd = torch.clamp(torch.sqrt(normv4 + (2 * gammav - torch.sqrt(gammav)) / vbarbar.max()) / (2 + normv2), max=1)
        t = exY * ip_yvbar - vbar * (ip_yvbar**2 + gammav) / 2
        b = -(1 - alphavd**2) * normv4 / gammav + 2 * alphavd**2
        H = torch.ones((d, 1), device=x.device) * 2 - (b + 2 * alphavd**2) * vbarbar
        invH = 1.0 / H
        s_step1 = yy - normv2 / gammav * (yvbar * ip_yvbar) - 1.0
        ip_vbart = vbar.T @ t
        s_step2 = s_step1 - alphavd / gammav * ((2 + normv2) * (t * vbar) - normv2 * vbarbar @ ip_vbart)
        invHvbarbar = invH * vbarbar
        ip_s = invHvbarbar.T @ s_step2
        s = (s_step2 * invH) - b / (1 + b * vbarbar.T @ invHvbarbar) * invHvbarbar @ ip_s
        ip_svbarbar = vbarbar.T @ s
        t = t - alphavd * ((2 + normv2) * (s * vbar) - vbar @ ip_svbarbar)
        exw = torch.cat([self.lrate_B * weights, weights[:1] * 0 + self.c1], 0)
        v = state.v + (t @ exw) / normv
        D = state.D + (s @ exw) * state.D
        nthroot = torch.exp(torch.log(D).sum() / d + torch.log(1 + v.T @ v) / (2 * d))[0, 0]
        D = D / nthroot
        G_s = ((z * z - 1.0) @ weights).sum() / d
        sigma = state.sigma * torch.exp(lrate_sigma / 2 * G_s)
        return state.update(p_sigma=p_sigma, center=center, p_c=p_c, v=v, D=D, sigma=sigma)
