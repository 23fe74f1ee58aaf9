"""Shared helpers of the ES zoo: optimiser sub-modules, sorting, device scalars."""
from __future__ import annotations

import torch

from ....utils import optim


def make_optimizer(optimizer, lr, center_init, **kw):
    """'adam' | 'sgd' | 'clipup' | a GradientTransformation | a Stateful → Stateful sub-module."""
    from ....core.module import Stateful

    if optimizer is None:
        return None
    if isinstance(optimizer, Stateful):
        return optimizer
    if isinstance(optimizer, str):
        if optimizer not in optim._BY_NAME:
            raise NotImplementedError(f"optimizer {optimizer!r}")
        optimizer = optim.get_optimizer(optimizer, learning_rate=lr, **kw)
    return optim.OptaxWrapper(optimizer, center_init)


def sort_by_key(keys: torch.Tensor, *vals: torch.Tensor):
    """Sort ``vals`` rows by ascending ``keys`` (reference ``sort_utils.py:5-12``)."""
    order = torch.argsort(keys, stable=True)
    return (keys[order],) + tuple(v[order] for v in vals)


def dscalar(x, device, dtype=torch.float32):
    return torch.as_tensor(x, dtype=dtype, device=device).clone()


def centered_ranks(fitness: torch.Tensor) -> torch.Tensor:
    n = fitness.shape[0]
    r = torch.empty(n, dtype=torch.float32, device=fitness.device)
    r[torch.argsort(fitness, stable=True)] = torch.arange(n, dtype=torch.float32, device=fitness.device)
    return r / (n - 1) - 0.5
