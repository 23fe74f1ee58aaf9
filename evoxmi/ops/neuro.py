"""Launcher of the persistent Ant + MLP rollout kernel (``neuro.hip``)."""
from __future__ import annotations

import torch

from . import _ext


def ant_param_count(h1: int, h2: int) -> int:
    return 27 * h1 + h1 + h1 * h2 + h2 + h2 * 8 + 8


def ant_rollout(flat_weights: torch.Tensor, h1: int, h2: int, init_state: torch.Tensor, cap: int):
    """Episode returns (N,) and lengths (N,) of N individuals whose MLP 27-h1-h2-8 (tanh)
    weights are rows of ``flat_weights`` in the layout [W1 (27×h1), b1, W2 (h1×h2), b2,
    W3 (h2×8), b3], all starting from ``init_state`` (29,)."""
    return _ext.ops().ant_rollout(flat_weights.to(torch.float32).contiguous(), int(h1), int(h2),
                                  init_state.to(device=flat_weights.device, dtype=torch.float32).contiguous(), int(cap))
