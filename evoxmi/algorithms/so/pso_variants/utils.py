"""PSO helpers (reference ``pso_variants/utils.py:8-60``)."""
from __future__ import annotations

import torch

from ....ops import random as rnd


def min_by(values, keys):
    if isinstance(values, (list, tuple)):
        values = torch.cat(list(values))
        keys = torch.cat(list(keys))
    i = torch.argmin(keys)
    return values.index_select(0, i.reshape(1))[0], keys.index_select(0, i.reshape(1))[0]


def get_distance_matrix(location: torch.Tensor) -> torch.Tensor:
    return torch.cdist(location, location)


def row_argsort(x: torch.Tensor) -> torch.Tensor:
    return torch.argsort(x, dim=-1, stable=True)


def select_from_mask(key, mask: torch.Tensor, s: int) -> torch.Tensor:
    """Random ``s`` positions among the nonzero entries of ``mask`` (1 = chosen)."""
    N = mask.shape[0]
    noise = rnd.uniform(key, (N,)).to(mask.device)
    idx = torch.argsort(mask.to(torch.float32) + noise, descending=True)
    idx = torch.where(torch.arange(N, device=mask.device) < s, idx, idx[max(s - 1, 0)])
    out = torch.zeros_like(mask)
    if s > 0:
        out[idx] = 1
    return out


def init_swarm(key_pop, key_v, pop_size, lb, ub, mean=None, stdev=None):
    dim = lb.shape[0]
    if mean is not None and stdev is not None:
        pop = torch.clamp(mean + stdev * rnd.normal(key_pop, (pop_size, dim)).to(lb.device), lb, ub)
        vel = stdev * rnd.normal(key_v, (pop_size, dim)).to(lb.device)
    else:
        length = ub - lb
        pop = rnd.uniform(key_pop, (pop_size, dim)).to(lb.device) * length + lb
        vel = rnd.uniform(key_v, (pop_size, dim)).to(lb.device) * length * 2 - length
    return pop, vel
