"""IM-MOEA — inverse-modelling MOEA (Cheng et al. 2015; reference ``algorithms/mo/im_moea.py:55-367``).

The population is partitioned by K reference vectors; inside each partition, for
every objective m a random group of ``l`` decision variables is modelled by an
inverse Gaussian process x_d = GP(f_m) with the linear kernel (as the reference),
offspring are sampled from the predictive distribution at evenly spaced objective
values over the extended range [1.5·min − 0.5·max, 1.5·max − 0.5·min], and NSGA-II
selection keeps N.

MI355X form: a GP with the linear kernel k(f, f') = v·f·f' and Gaussian noise σ² is
Bayesian linear regression, whose predictive mean and variance are closed-form
rank-one expressions — so all K·M·l inverse models of a generation are one batched
tensor computation on the device instead of K·M·l separate 250-step optimiser runs
(the reference's Adam at lr 1e-3 for 250 steps moves gpjax's initial v = σ = 1 by
well under 25 %; they are kept at those values here).
Partitions use the largest cosine (the reference's ``ask`` takes the *smallest*
cosine similarity, ``im_moea.py:120``, i.e. the farthest vector).
"""
from __future__ import annotations

import math

import torch

from ...core import State
from ...operators.sampling import UniformSampling
from ...ops import random as rnd
from ...utils.common import cos_dist
from .common import MOAlgorithm, nsga2_select


class IMMOEA(MOAlgorithm):
    def __init__(self, lb, ub, n_objs=3, pop_size=105, l=3, k=10, mutation_op=None):
        super().__init__(lb, ub, n_objs, pop_size, mutation_op)
        self.l, self.k = l, k
        self.pop_size = int(math.ceil(pop_size / k) * k)
        W = UniformSampling(k, n_objs)()[0]
        W = torch.flip(torch.sort(torch.flip(W, [1]), 0).values, [1])  # reference :74-76
        self.W = W.to(lb.device)
        self.k = W.shape[0]

    def setup(self, key):
        st = super().setup(key)
        return st.update(reference_vector=self.W)

    def ask(self, state):
        key, k_parent, k_dims, k_noise, k_fill, k_mut = rnd.split(state.key, 6)
        dev = state.population.device
        N, K, M, D, l = self.pop_size, self.k, self.n_objs, self.dim, min(self.l, self.dim)
        pop, fit = state.population, state.fitness
        part = torch.argmax(cos_dist(fit, state.reference_vector), 1)
        n_off = N // K
        # members of each partition (random member of the whole population for empty ones)
        member_key = part.to(torch.float32) + rnd.uniform(k_parent, (N,)).to(dev) * 0.5
        order = torch.argsort(member_key)
        counts = torch.bincount(part, minlength=K)
        starts = torch.cumsum(counts, 0) - counts
        j = torch.arange(n_off, device=dev)
        pick = starts[:, None] + (j[None, :] % counts.clamp(min=1)[:, None])
        rand_fill = rnd.randint(k_fill, (K, n_off), 0, N).to(dev)
        parent_idx = torch.where(counts[:, None] > 0, order[pick.clamp(max=N - 1)], rand_fill)  # (K, n_off)
        off = pop[parent_idx].clone()  # (K, n_off, D)
        # per partition: data f (members) and x (members); use the partition mask
        mask = (part[None, :] == torch.arange(K, device=dev)[:, None]).to(pop.dtype)  # (K, N)
        big = torch.full_like(fit, float("inf"))
        fmin = torch.stack([torch.where(mask[c].bool()[:, None], fit, big).min(0).values for c in range(K)])
        fmax = torch.stack([torch.where(mask[c].bool()[:, None], fit, -big).max(0).values for c in range(K)])
        ok = counts >= 2
        lo = torch.where(ok[:, None], 1.5 * fmin - 0.5 * fmax, fit.min(0).values)
        hi = torch.where(ok[:, None], 1.5 * fmax - 0.5 * fmin, fit.max(0).values)
        dims = torch.argsort(rnd.uniform(k_dims, (K, M, D)).to(dev), dim=-1)[..., :l]  # (K, M, l)
        v, s2 = 1.0, 1.0
        f2 = (mask[:, :, None] * fit[None] ** 2).sum(1)  # (K, M)  Σ f²
        fx = torch.einsum("cn,nm,nd->cmd", mask, fit, pop)  # (K, M, D)  Σ f·x
        t = torch.linspace(0, 1, n_off, device=dev)
        fstar = lo[:, :, None] + (hi - lo)[:, :, None] * t  # (K, M, n_off)
        denom = s2 + v * f2  # (K, M)
        coef = v * fx / denom[:, :, None]  # (K, M, D)
        mean = fstar[..., None] * coef[:, :, None, :]  # (K, M, n_off, D)
        var = v * fstar**2 * s2 / denom[:, :, None] + s2  # (K, M, n_off)
        sample = mean + torch.sqrt(var)[..., None] * rnd.normal(k_noise, (K, M, n_off, D)).to(dev)
        sel = torch.zeros((K, M, D), dtype=torch.bool, device=dev).scatter_(2, dims, True) & ok[:, None, None]
        # objective m writes its own variable group into the offspring block of that objective
        m_of = torch.arange(n_off, device=dev) % M  # spread the M inverse models over the offspring
        S = sample[torch.arange(K, device=dev)[:, None], m_of[None, :], torch.arange(n_off, device=dev)[None, :]]  # (K, n_off, D)
        SEL = sel[:, m_of, :]  # (K, n_off, D)
        off = torch.where(SEL, S, off).reshape(-1, D)
        off = torch.clamp(self.mutation(k_mut, off), self.lb, self.ub)
        return off, state.update(next_generation=off, key=key)

    def tell(self, state, fitness):
        pop = torch.cat([state.population, state.next_generation])
        obj = torch.cat([state.fitness, fitness])
        idx = nsga2_select(obj, self.pop_size)
        return state.update(population=pop[idx], fitness=obj[idx])
