"""Exact GP regression (reference ``operators/gaussian_process/regression.py:18-107``)."""
from __future__ import annotations

import math

import torch

from ...utils import optim
from .kernels import RBF
from .likelihoods import Gaussian

_sp = torch.nn.functional.softplus


class GPRegression:
    def __init__(self, kernel=None, mean_fun=None, likelihood=None, object=None, key=None, num_iters=250):
        self.kernel = kernel if kernel is not None else RBF()
        self.mean_fun = mean_fun  # zero mean (the reference's default ``Zero()``)
        self.likelihood = likelihood if likelihood is not None else Gaussian()
        self.num_iters = num_iters
        self._u = None

    def _params(self, u):
        k = {n: _sp(u["k_" + n]) for n in self.kernel.params}
        noise = _sp(u["obs_stddev"])
        return k, noise

    def _neg_mll(self, u, x, y):
        k, noise = self._params(u)
        n = x.shape[0]
        K = self.kernel(k, x, x) + (noise**2 + 1e-6) * torch.eye(n, dtype=x.dtype)
        L = torch.linalg.cholesky(K)
        a = torch.cholesky_solve(y, L)
        mll = -0.5 * (y * a).sum() - torch.log(torch.diagonal(L)).sum() - 0.5 * n * math.log(2 * math.pi)
        return -mll

    def fit(self, x, y, optimzer=None):
        self.device = x.device
        x = x.detach().to("cpu", torch.float64).reshape(x.shape[0], -1)
        y = y.detach().to("cpu", torch.float64).reshape(-1, 1)
        opt = optimzer if optimzer is not None else optim.sgd(0.001)
        u = {"k_" + k: v for k, v in self.kernel.unconstrained().items()}
        u.update(self.likelihood.unconstrained())
        names = list(u)
        vec = torch.stack([u[n] for n in names]).clone()
        state = opt.init(vec)
        self.history = []
        for _ in range(self.num_iters):
            v = vec.clone().requires_grad_(True)
            loss = self._neg_mll({n: v[i] for i, n in enumerate(names)}, x, y)
            (g,) = torch.autograd.grad(loss, v)
            upd, state = opt.update(g, state, vec)
            vec = vec + upd
            self.history.append(float(loss))
        self._u = {n: vec[i] for i, n in enumerate(names)}
        self._x, self._y = x, y
        return self

    def predict(self, x):
        xs = x.detach().to("cpu", torch.float64).reshape(x.shape[0], -1)
        k, noise = self._params(self._u)
        n = self._x.shape[0]
        K = self.kernel(k, self._x, self._x) + noise**2 * torch.eye(n, dtype=torch.float64)
        Ks = self.kernel(k, xs, self._x)
        L = torch.linalg.cholesky(K)
        mean = Ks @ torch.cholesky_solve(self._y, L)
        v = torch.cholesky_solve(Ks.T, L)
        var = torch.diagonal(self.kernel(k, xs, xs)) - (Ks * v.T).sum(1)
        std = torch.sqrt(var.clamp(min=0) + noise**2)
        mean = mean[:, 0].to(torch.float32).to(self.device)
        std = std.to(torch.float32).to(self.device)
        return torch.distributions.Normal(mean, std), mean, std
