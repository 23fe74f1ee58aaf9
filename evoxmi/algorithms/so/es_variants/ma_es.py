"""MA-ES and LM-MA-ES.

Reference: ``es_variants/ma_es.py:24-126``.  The reference's versions plug M into
the CMA-ES formulas where C and C^{-1/2} belong (``ps ← … M Δm``, ``M ← (1−c1−cμ)M +
c1 p pᵀ + cμ Σ w y yᵀ``), which is neither MA-ES nor convergent (on the 5-D sphere
of the test protocol it stalls at f ≈ 10²).  These are the published algorithms:

* MA-ES (Beyer & Sendhoff 2017): ``d = M z``, ``s ← (1−cs)s + √(cs(2−cs)μ_eff)·⟨z⟩_w``,
  ``M ← M[I + c1/2 (s sᵀ − I) + cμ/2 (⟨z zᵀ⟩_w − I)]`` — no eigendecomposition,
  one (d×d)·(d×d) GEMM per generation;
* LM-MA-ES (Loshchilov, Glasmachers & Beyer 2017): m direction vectors with
  learning rates ``c_d,j = 1/(1.5^(j−1) n)``, ``c_c,j = λ/(4^(j−1) n)``; sampling
  applies the m rank-one contractions to z (O(m·λ·n)), no n×n matrix at all.
"""
from __future__ import annotations

import math

import torch

from ....core import State
from ....ops import random as rnd
from ._cma_base import TextbookCMA


class MAES(TextbookCMA):
    def setup(self, key):
        dev = self.center_init.device
        d = self.dim
        return State(ps=torch.zeros(d, device=dev), M=torch.eye(d, device=dev), count_iter=torch.zeros((), dtype=torch.int64, device=dev),
                     mean=self.center_init.to(torch.float32).clone(), sigma=torch.tensor(self.init_stdev, dtype=torch.float32, device=dev),
                     key=key.to(dev), population=torch.zeros((self.pop_size, d), device=dev), noise=torch.zeros((self.pop_size, d), device=dev))

    def ask(self, state):
        key, sample_key = rnd.split(state.key)
        z = rnd.normal(sample_key, (self.pop_size, self.dim)).to(state.mean.device)
        population = state.mean + state.sigma * z @ state.M.T
        return population, state.update(population=population, noise=z, count_iter=state.count_iter + 1, key=key)

    def _sigma(self, sigma, ps):
        return sigma * torch.exp((self.cs / self.damps) * (torch.linalg.norm(ps) / self.chiN - 1))

    def tell(self, state, fitness):
        order = torch.argsort(fitness, stable=True)[: self.mu]
        z = state.noise[order]
        x = state.population[order]
        w = self.weights
        zw = w @ z
        mean = w @ x
        ps = (1 - self.cs) * state.ps + math.sqrt(self.cs * (2 - self.cs) * self.mueff) * zw
        I = torch.eye(self.dim, device=z.device)
        G = self.c1 / 2 * (torch.outer(ps, ps) - I) + self.cmu / 2 * ((z.T * w) @ z - I)
        M = state.M + state.M @ G
        return state.update(mean=mean, ps=ps, M=M, sigma=self._sigma(state.sigma, ps))


class LMMAES(TextbookCMA):
    def __init__(self, *args, memory_size=None, **kwargs):
        super().__init__(*args, **kwargs)
        n = self.dim
        self.memory_size = memory_size or (4 + int(3 * math.log(n)))
        j = torch.arange(self.memory_size, dtype=torch.float32)
        self.c_d = (1.0 / (1.5**j * n)).to(self.center_init.device)
        self.c_c = (self.pop_size / (4.0**j * n)).clamp(max=1.0).to(self.center_init.device)
        self.c_s = 2 * self.pop_size / n if 2 * self.pop_size < n else 0.3  # paper: c_σ = 2λ/n

    def setup(self, key):
        dev = self.center_init.device
        d = self.dim
        return State(ps=torch.zeros(d, device=dev), Mv=torch.zeros((self.memory_size, d), device=dev),
                     count_iter=torch.zeros((), dtype=torch.int64, device=dev), mean=self.center_init.to(torch.float32).clone(),
                     sigma=torch.tensor(self.init_stdev, dtype=torch.float32, device=dev), key=key.to(dev),
                     population=torch.zeros((self.pop_size, d), device=dev), noise=torch.zeros((self.pop_size, d), device=dev),
                     dvec=torch.zeros((self.pop_size, d), device=dev))

    def ask(self, state):
        key, sample_key = rnd.split(state.key)
        z = rnd.normal(sample_key, (self.pop_size, self.dim)).to(state.mean.device)
        d = z
        active = torch.arange(self.memory_size, device=z.device) < state.count_iter  # j ≤ min(t, m)
        for j in range(self.memory_size):
            mj = state.Mv[j]
            upd = (1 - self.c_d[j]) * d + self.c_d[j] * (d @ mj)[:, None] * mj[None, :]
            d = torch.where(active[j], upd, d)
        population = state.mean + state.sigma * d
        return population, state.update(population=population, noise=z, dvec=d, count_iter=state.count_iter + 1, key=key)

    def tell(self, state, fitness):
        order = torch.argsort(fitness, stable=True)[: self.mu]
        w = self.weights
        zw = w @ state.noise[order]
        mean = state.mean + state.sigma * (w @ state.dvec[order])
        cs = self.c_s
        ps = (1 - cs) * state.ps + math.sqrt(cs * (2 - cs) * self.mueff) * zw
        Mv = (1 - self.c_c)[:, None] * state.Mv + torch.sqrt(self.mueff * self.c_c * (2 - self.c_c))[:, None] * zw[None, :]
        sigma = state.sigma * torch.exp(cs / 2 * ((ps * ps).sum() / self.dim - 1))
        return state.update(mean=mean, ps=ps, Mv=Mv, sigma=sigma)
