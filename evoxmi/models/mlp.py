"""Batched per-individual MLP policies.

``MLPPolicy(sizes)`` plays the role of the reference tests' flax modules:
``init(key) -> params`` (a dict pytree, usable with :class:`~evoxmi.utils.TreeAndVector`)
and ``apply(params, obs)`` where every leaf of ``params`` has a leading population
axis and ``obs`` is (N, in) — one ``torch.bmm`` per layer (batched GEMM on the
matrix cores).  ``flat(params)`` gives the [W1, b1, W2, b2, …] row layout consumed
by the fused rollout kernels.
"""
from __future__ import annotations

import math

import torch

from ..ops import random as rnd

_ACT = {"tanh": torch.tanh, "relu": torch.relu, "sigmoid": torch.sigmoid, "identity": lambda x: x, None: lambda x: x}


class MLPPolicy:
    def __init__(self, sizes, activation="tanh", output_activation="tanh", discrete=False):
        self.sizes = list(sizes)
        self.activation = activation
        self.output_activation = output_activation
        self.discrete = discrete

    def init(self, key, device=None):
        params = {}
        keys = rnd.split(key, len(self.sizes) - 1)
        for i, (a, b) in enumerate(zip(self.sizes[:-1], self.sizes[1:])):
            lim = math.sqrt(6.0 / (a + b))  # Glorot-uniform, flax Dense's default initialiser family
            params[f"layer{i}"] = {"w": (rnd.uniform(keys[i], (a, b)) * 2 - 1).to(device) * lim, "b": torch.zeros(b, device=device)}
        return params

    @property
    def num_params(self):
        return sum(a * b + b for a, b in zip(self.sizes[:-1], self.sizes[1:]))

    def apply(self, params, obs):
        """Batched forward: params leaves (N, …), obs (N, in) → (N, out)."""
        x = obs
        n = len(self.sizes) - 1
        for i in range(n):
            p = params[f"layer{i}"]
            w, b = p["w"], p["b"]
            if w.dim() == 2:  # unbatched parameters (one policy for all)
                x = x @ w + b
            else:
                x = torch.bmm(x[:, None, :], w)[:, 0, :] + b
            x = _ACT[self.activation if i < n - 1 else self.output_activation](x)
        return x

    __call__ = apply

    def flat(self, params):
        """[W1, b1, W2, b2, …] rows (N, P) — the fused-kernel layout."""
        parts = []
        for i in range(len(self.sizes) - 1):
            p = params[f"layer{i}"]
            n = p["w"].shape[0]
            parts += [p["w"].reshape(n, -1), p["b"].reshape(n, -1)]
        return torch.cat(parts, 1)
