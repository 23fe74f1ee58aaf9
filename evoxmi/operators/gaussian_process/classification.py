"""GP classification with a Bernoulli (probit) likelihood
(reference ``operators/gaussian_process/classification.py:16-102``, gpjax ``LogPosteriorDensity``).

MAP estimate of the whitened latent values f = L v jointly with the kernel
hyper-parameters (500 Adam steps by default); predictions condition the latent GP
on the MAP values and return the probit predictive Bernoulli mean Φ(μ/√(1+σ²)).
Parity unpinned: no reference fixture exists for classification.
"""
from __future__ import annotations

import math

import torch

from ...utils import optim
from .kernels import RBF

_sp = torch.nn.functional.softplus


def _log_phi(z):
    return torch.special.log_ndtr(z)


class GPClassification:
    def __init__(self, kernel=None, mean_fun=None, likelihood=None, object=None, key=None, num_iters=500):
        self.kernel = kernel if kernel is not None else RBF()
        self.likelihood = likelihood
        self.num_iters = num_iters

    def fit(self, x, y, optimizer=None):
        self.device = x.device
        x = x.detach().to("cpu", torch.float64).reshape(x.shape[0], -1)
        y = y.detach().to("cpu", torch.float64).reshape(-1)
        n = x.shape[0]
        opt = optimizer if isinstance(optimizer, optim.GradientTransformation) else optim.adam(0.01)
        ku = self.kernel.unconstrained()
        names = list(ku)
        vec = torch.cat([torch.stack([ku[k] for k in names]), torch.zeros(n, dtype=torch.float64)])
        state = opt.init(vec)
        s = 2 * y - 1
        for _ in range(self.num_iters):
            v = vec.clone().requires_grad_(True)
            p = {k: _sp(v[i]) for i, k in enumerate(names)}
            K = self.kernel(p, x, x) + 1e-6 * torch.eye(n, dtype=torch.float64)
            L = torch.linalg.cholesky(K)
            f = L @ v[len(names):]
            logpost = _log_phi(s * f).sum() - 0.5 * (v[len(names):] ** 2).sum()
            (g,) = torch.autograd.grad(-logpost, v)
            upd, state = opt.update(g, state, vec)
            vec = vec + upd
        self._p = {k: _sp(vec[i]) for i, k in enumerate(names)}
        self._x = x
        K = self.kernel(self._p, x, x) + 1e-6 * torch.eye(n, dtype=torch.float64)
        self._L = torch.linalg.cholesky(K)
        self._f = self._L @ vec[len(names):]
        return self

    def predict(self, x):
        xs = x.detach().to("cpu", torch.float64).reshape(x.shape[0], -1)
        Ks = self.kernel(self._p, xs, self._x)
        alpha = torch.cholesky_solve(self._f[:, None], self._L)
        mu = (Ks @ alpha)[:, 0]
        v = torch.cholesky_solve(Ks.T, self._L)
        var = (torch.diagonal(self.kernel(self._p, xs, xs)) - (Ks * v.T).sum(1)).clamp(min=0)
        prob = torch.special.ndtr(mu / torch.sqrt(1 + var))
        prob = prob.to(torch.float32).to(self.device)
        return torch.distributions.Bernoulli(probs=prob), prob, torch.sqrt(prob * (1 - prob))
