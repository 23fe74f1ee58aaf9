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
        """[W1, b1, W2, b2, …] rows (N, P) — the fused-kernel layout.  When the leaves are
        consecutive column slices of one row-major (N, P) buffer (what
        ``TreeAndVector.batched_to_tree`` produces from the population), that buffer is
        returned as a view instead of being copied (212 MB per generation at the
        north-star shape)."""
        parts = []
        for i in range(len(self.sizes) - 1):
            p = params[f"layer{i}"]
            n = p["w"].shape[0]
            parts += [p["w"].reshape(n, -1), p["b"].reshape(n, -1)]
        base = _contiguous_columns(parts)
        return base if base is not None else torch.cat(parts, 1)


def _contiguous_columns(parts):
    """The (N, ΣP) view covering ``parts`` if they are adjacent column blocks of one buffer."""
    p0 = parts[0]
    P = sum(t.shape[1] for t in parts)
    ptr = p0.untyped_storage().data_ptr()
    off = p0.storage_offset()
    for t in parts:
        if t.untyped_storage().data_ptr() != ptr or t.storage_offset() != off or (t.shape[0] > 1 and t.stride(0) != P) or t.stride(1) != 1:
            return None
        off += t.shape[1]
    return p0.as_strided((p0.shape[0], P), (P, 1), p0.storage_offset())
