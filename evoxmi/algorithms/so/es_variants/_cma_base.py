"""Textbook CMA-ES update rules as overridable methods — the base of the CMA-derived
variants (MA-ES, LM-MA-ES, RM-ES, AMaLGaM), mirroring the helper structure of the
reference's ``cma_es.py:104-136`` (``_update_mean/_update_ps/_update_pc/_update_C/
_update_sigma/_decomposition_C``).  Sampling, state layout and the (warm-started
Jacobi, graph-capturable) eigendecomposition are those of :class:`CMAES`.
"""
from __future__ import annotations

import torch

from .cma_es import CMAES
from ._common import sort_by_key


class TextbookCMA(CMAES):
    def _update_mean(self, mean, population):
        return mean + self.cm * (self.weights @ (population[: self.mu] - mean))

    def _update_ps(self, ps, invsqrtC, sigma, delta_mean):
        return (1 - self.cs) * ps + (self.cs * (2 - self.cs) * self.mueff) ** 0.5 * (invsqrtC @ delta_mean) / sigma

    def _update_pc(self, pc, ps, delta_mean, sigma, hsig):
        return (1 - self.cc) * pc + hsig * (self.cc * (2 - self.cc) * self.mueff) ** 0.5 * delta_mean / sigma

    def _update_C(self, C, pc, sigma, population, old_mean, hsig):
        y = (population[: self.mu] - old_mean) / sigma
        return ((1 - self.c1 - self.cmu) * C + self.c1 * (torch.outer(pc, pc) + (1 - hsig) * self.cc * (2 - self.cc) * C)
                + self.cmu * (y.T * self.weights) @ y)

    def _update_sigma(self, sigma, ps):
        return sigma * torch.exp((self.cs / self.damps) * (torch.linalg.norm(ps) / self.chiN - 1))

    def _hsig(self, ps, count_iter):
        return (torch.linalg.norm(ps) / torch.sqrt(1 - (1 - self.cs) ** (2 * count_iter.to(torch.float32)))
                < (1.4 + 2 / (self.dim + 1)) * self.chiN).to(torch.float32)

    def _decompose_every(self, state, C):
        B, D, invsqrtC = self._decomposition_C(C, state.B)
        if self.decomp_per_iter > 1:
            do = (state.count_iter % self.decomp_per_iter) == 0
            B, D, invsqrtC = (torch.where(do, a, b) for a, b in ((B, state.B), (D, state.D), (invsqrtC, state.invsqrtC)))
        return B, D, invsqrtC

    def tell(self, state, fitness):
        _, population = sort_by_key(fitness, state.population)
        mean = self._update_mean(state.mean, population)
        delta_mean = mean - state.mean
        ps = self._update_ps(state.ps, state.invsqrtC, state.sigma, delta_mean)
        hsig = self._hsig(ps, state.count_iter)
        pc = self._update_pc(state.pc, ps, delta_mean, state.sigma, hsig)
        C = self._update_C(state.C, pc, state.sigma, population, state.mean, hsig)
        sigma = self._update_sigma(state.sigma, ps)
        B, D, invsqrtC = self._decompose_every(state, C)
        return state.update(mean=mean, ps=ps, pc=pc, C=C, sigma=sigma, B=B, D=D, invsqrtC=invsqrtC)
