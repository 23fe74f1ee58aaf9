"""IM-MOEA — inverse-modelling MOEA (Cheng et al. 2015; reference ``algorithms/mo/im_moea.py:55-367``).

The population is partitioned by K reference vectors; inside each partition, for
every objective m a random group of ``l`` decision variables is modelled by an
inverse Gaussian process x_d = GP(f_m) with the linear kernel (as the reference),
offspring are sampled from the predictive distribution at evenly spaced objective
values over the extended range [1.5·min − 0.5·max, 1.5·max − 0.5·min], and NSGA-II
selection keeps N.

MI355X form: a GP with the linear kernel k(f, f') = v·f·f' and Gaussian noise s² is
Bayesian linear regression: its marginal likelihood and predictive mean / variance are
closed-form in the sufficient statistics (Σf², Σf·x, Σx², n).  The hyper-parameters are
fitted as in the reference (250 Adam steps at lr 1e-3 on the softplus-unconstrained
(v, s) from v = s = 1, ``im_moea.py:310-314``) for every partition × objective × variable
at once: one thread per model runs the whole optimisation in registers
(``csrc/kernels/gp_fit.hip``; :func:`linear_gp_fit` is the torch reference), then all
inverse models are sampled in one batched tensor computation.
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


_U0 = 0.5413248546129181  # softplus⁻¹(1)


def linear_gp_fit(a, b, c, n, steps: int = 250, lr: float = 1e-3):
    """(v, s²) of linear-kernel GP regressions x = GP(f) from the sufficient statistics
    a = Σf², b = Σf·x, c = Σx², n (tensors of one shape): Adam on the negative marginal
    likelihood nll = ½(c − v b²/D)/s² + ½(n − 1) log s² + ½ log D, D = s² + v a, in softplus
    coordinates (the reference's gpjax ``Linear`` kernel + ``Gaussian`` likelihood fit)."""
    a, b, c, n = (t.to(torch.float64).contiguous() for t in (a, b, c, n))
    if a.is_cuda:
        from ...ops import _ext

        return tuple(_ext.ops().linear_gp_fit(a, b, c, n, int(steps), float(lr)))
    sp = torch.nn.functional.softplus
    uv = torch.full_like(a, _U0)
    us = torch.full_like(a, _U0)
    mv, ms, vv, vs = (torch.zeros_like(a) for _ in range(4))
    for t in range(1, steps + 1):
        v, s = sp(uv), sp(us)
        s2 = s * s
        D = s2 + v * a
        gv = -0.5 * b * b / (D * D) + 0.5 * a / D
        gs2 = -0.5 * c / (s2 * s2) + 0.5 * v * b * b * (s2 + D) / (D * D * s2 * s2) + 0.5 * (n - 1) / s2 + 0.5 / D
        g_uv, g_us = gv * torch.sigmoid(uv), gs2 * 2 * s * torch.sigmoid(us)
        mv, ms = 0.9 * mv + 0.1 * g_uv, 0.9 * ms + 0.1 * g_us
        vv, vs = 0.999 * vv + 0.001 * g_uv * g_uv, 0.999 * vs + 0.001 * g_us * g_us
        uv = uv - lr * (mv / (1 - 0.9**t)) / (torch.sqrt(vv / (1 - 0.999**t)) + 1e-8)
        us = us - lr * (ms / (1 - 0.9**t)) / (torch.sqrt(vs / (1 - 0.999**t)) + 1e-8)
    s = sp(us)
    return sp(uv).float(), (s * s).float()


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
        f2 = (mask[:, :, None] * fit[None] ** 2).sum(1)  # (K, M)  Σ f²
        fx = torch.einsum("cn,nm,nd->cmd", mask, fit, pop)  # (K, M, D)  Σ f·x
        xx = mask @ (pop * pop)  # (K, D)  Σ x²
        # fitted hyper-parameters of every (partition, objective, variable) inverse model
        v, s2 = linear_gp_fit(f2[:, :, None].expand(K, M, D), fx, xx[:, None, :].expand(K, M, D),
                              counts.to(torch.float64)[:, None, None].expand(K, M, D))
        v, s2 = v.to(pop.dtype), s2.to(pop.dtype)
        t = torch.linspace(0, 1, n_off, device=dev)
        fstar = lo[:, :, None] + (hi - lo)[:, :, None] * t  # (K, M, n_off)
        denom = s2 + v * f2[:, :, None]  # (K, M, D)
        coef = v * fx / denom  # (K, M, D)
        mean = fstar[..., None] * coef[:, :, None, :]  # (K, M, n_off, D)
        var = (v * s2 / denom)[:, :, None, :] * (fstar**2)[..., None] + s2[:, :, None, :]  # (K, M, n_off, D)
        sample = mean + torch.sqrt(var) * rnd.normal(k_noise, (K, M, n_off, D)).to(dev)
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
