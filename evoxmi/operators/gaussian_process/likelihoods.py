"""Observation models."""
from __future__ import annotations

import torch

from .kernels import softplus_inv


class Gaussian:
    def __init__(self, num_datapoints=None, obs_stddev=1.0):
        self.num_datapoints = num_datapoints
        self.params = {"obs_stddev": float(obs_stddev)}

    def unconstrained(self):
        return {k: torch.tensor(softplus_inv(v), dtype=torch.float64) for k, v in self.params.items()}


class Bernoulli:
    """Probit link: p(y = 1 | f) = Φ(f)."""

    def __init__(self, num_datapoints=None):
        self.num_datapoints = num_datapoints
        self.params = {}

    def unconstrained(self):
        return {}
