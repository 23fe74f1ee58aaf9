"""Covariance functions with softplus-constrained parameters."""
from __future__ import annotations

import math

import torch


def softplus_inv(v: float) -> float:
    return math.log(math.expm1(v)) if v < 20 else v


class Kernel:
    params: dict

    def unconstrained(self):
        return {k: torch.tensor(softplus_inv(v), dtype=torch.float64) for k, v in self.params.items()}

    @staticmethod
    def constrain(u):
        return {k: torch.nn.functional.softplus(v) for k, v in u.items()}


class RBF(Kernel):
    def __init__(self, lengthscale=1.0, variance=1.0):
        self.params = {"lengthscale": float(lengthscale), "variance": float(variance)}

    def __call__(self, p, x, y):
        d2 = ((x[:, None, :] - y[None, :, :]) ** 2).sum(-1)
        return p["variance"] * torch.exp(-0.5 * d2 / p["lengthscale"] ** 2)


class Matern52(Kernel):
    def __init__(self, lengthscale=1.0, variance=1.0):
        self.params = {"lengthscale": float(lengthscale), "variance": float(variance)}

    def __call__(self, p, x, y):
        r = torch.sqrt(((x[:, None, :] - y[None, :, :]) ** 2).sum(-1).clamp(min=1e-36)) / p["lengthscale"]
        s5 = math.sqrt(5.0)
        return p["variance"] * (1 + s5 * r + 5.0 / 3.0 * r * r) * torch.exp(-s5 * r)


class Linear(Kernel):
    def __init__(self, variance=1.0):
        self.params = {"variance": float(variance)}

    def __call__(self, p, x, y):
        return p["variance"] * (x @ y.T)
