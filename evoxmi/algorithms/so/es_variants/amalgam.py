"""AMaLGaM and IndependentAMaLGaM (reference ``es_variants/amalgam.py:22-133``).

CMA-ES with an anticipated mean shift (``m + α σ p_c``) and adaptive variance
scaling by the standard-deviation ratio of the best sample.  The reference's
``_update_C`` uses the 5-argument ``lax.cond`` removed from JAX (``amalgam.py:38``)
and therefore raises; here the scaling is applied to the *updated* covariance, the
evident intent.  The standard-deviation ratio of the best sample is measured in
units of the current distribution (‖y₀‖/√d, resp. |y₀| per coordinate, with
y = (x − m)/σ) — the reference divides by σ a second time, which makes the ratio
explode as σ shrinks and the covariance overflow.
"""
from __future__ import annotations

import torch

from ....core import State
from ....ops import random as rnd
from ._cma_base import TextbookCMA
from ._common import sort_by_key

ALPHA, BETA = 0.05, 0.05


class AMaLGaM(TextbookCMA):
    def _update_mean_shift(self, mean, population, sigma, pc):
        return self._update_mean(mean, population) + ALPHA * sigma * pc

    def _update_C(self, C, pc, sigma, population, old_mean, hsig):
        updated = super()._update_C(C, pc, sigma, population, old_mean, hsig)
        y = (population[: self.mu] - old_mean) / sigma
        sdr = torch.linalg.norm(y[0]) / self.dim**0.5
        return torch.where(sdr > 1, (1 + BETA * (sdr - 1)) * updated, updated / (1 + BETA * (1 - sdr)))

    def tell(self, state, fitness):
        _, population = sort_by_key(fitness, state.population)
        mean = self._update_mean_shift(state.mean, population, state.sigma, state.pc)
        delta_mean = mean - state.mean
        ps = self._update_ps(state.ps, state.invsqrtC, state.sigma, delta_mean)
        hsig = self._hsig(ps, state.count_iter)
        pc = self._update_pc(state.pc, ps, delta_mean, state.sigma, hsig)
        C = self._update_C(state.C, pc, state.sigma, population, state.mean, hsig)
        sigma = self._update_sigma(state.sigma, ps)
        B, D, invsqrtC = self._decompose_every(state, C)
        return state.update(mean=mean, ps=ps, pc=pc, C=C, sigma=sigma, B=B, D=D, invsqrtC=invsqrtC)


class IndependentAMaLGaM(AMaLGaM):
    """Diagonal-covariance AMaLGaM (per-coordinate variance and SDR)."""

    def setup(self, key):
        dev = self.center_init.device
        d = self.dim
        return State(pc=torch.zeros(d, device=dev), ps=torch.zeros(d, device=dev), C=torch.ones(d, device=dev),
                     count_iter=torch.zeros((), dtype=torch.int64, device=dev), mean=self.center_init.to(torch.float32).clone(),
                     sigma=torch.tensor(self.init_stdev, dtype=torch.float32, device=dev), key=key.to(dev),
                     population=torch.zeros((self.pop_size, d), device=dev))

    def _update_C(self, C, pc, sigma, population, old_mean, hsig):
        y = (population[: self.mu] - old_mean) / sigma
        sdr = torch.abs(y[0])
        C = (1 - self.c1 - self.cmu) * C + self.c1 * (pc**2 + (1 - hsig) * self.cc * (2 - self.cc) * C) + self.cmu * (self.weights @ (y**2))
        return torch.where(sdr > 1, (1 + BETA * (sdr - 1)) * C, C / (1 + BETA * (1 - sdr)))

    def ask(self, state):
        key, sample_key = rnd.split(state.key)
        noise = rnd.normal(sample_key, (self.pop_size, self.dim)).to(state.mean.device)
        population = state.mean + state.sigma * (torch.sqrt(state.C) * noise)
        return population, state.update(population=population, count_iter=state.count_iter + 1, key=key)

    def tell(self, state, fitness):
        _, population = sort_by_key(fitness, state.population)
        mean = self._update_mean_shift(state.mean, population, state.sigma, state.pc)
        delta_mean = mean - state.mean
        # the reference passes the diagonal C where invsqrtC belongs (amalgam.py:120), and
        # ``C @ Δm`` of two vectors is a dot product there; the diagonal C^{-1/2} Δm is used here
        ps = (1 - self.cs) * state.ps + (self.cs * (2 - self.cs) * self.mueff) ** 0.5 * (delta_mean / torch.sqrt(state.C)) / state.sigma
        hsig = self._hsig(ps, state.count_iter)
        pc = self._update_pc(state.pc, ps, delta_mean, state.sigma, hsig)
        C = self._update_C(state.C, pc, state.sigma, population, state.mean, hsig)
        sigma = self._update_sigma(state.sigma, ps)
        return state.update(mean=mean, ps=ps, pc=pc, C=C, sigma=sigma)
