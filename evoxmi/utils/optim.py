"""Functional first-order optimisers with state held in the :class:`State` tree.

The reference wraps optax optimisers as a Stateful sub-module (``OptaxWrapper``,
``src/evox/utils/common.py:149-161``) and ships ClipUp (``pgpe.py:29``).  optax is
a JAX library, so evoxmi provides the same functional contract natively:
``opt.init(params) -> opt_state`` and ``opt.update(grads, opt_state, params) ->
(updates, opt_state)`` where ``params + updates`` is the new point.
"""
from __future__ import annotations

import math
from typing import Any, NamedTuple

import torch

from ..core.module import Stateful
from ..core.state import State


class GradientTransformation(NamedTuple):
    init: Any
    update: Any


def sgd(learning_rate: float, momentum: float = 0.0, nesterov: bool = False) -> GradientTransformation:
    def init(params):
        return (torch.zeros_like(params),) if momentum else ()

    def update(grads, opt_state, params=None):
        if not momentum:
            return -learning_rate * grads, opt_state
        (v,) = opt_state
        v = momentum * v + grads
        g = grads + momentum * v if nesterov else v
        return -learning_rate * g, (v,)

    return GradientTransformation(init, update)


def adam(learning_rate: float, b1: float = 0.9, b2: float = 0.999, eps: float = 1e-8, weight_decay: float = 0.0) -> GradientTransformation:
    def init(params):
        z = torch.zeros_like(params)
        return (torch.zeros((), dtype=torch.float32, device=params.device), z, z.clone())

    def update(grads, opt_state, params=None):
        t, m, v = opt_state
        t = t + 1
        m = b1 * m + (1 - b1) * grads
        v = b2 * v + (1 - b2) * grads * grads
        mhat = m / (1 - b1**t)
        vhat = v / (1 - b2**t)
        upd = -learning_rate * mhat / (torch.sqrt(vhat) + eps)
        if weight_decay and params is not None:
            upd = upd - learning_rate * weight_decay * params
        return upd, (t, m, v)

    return GradientTransformation(init, update)


def adamw(learning_rate: float, b1=0.9, b2=0.999, eps=1e-8, weight_decay=1e-4):
    return adam(learning_rate, b1, b2, eps, weight_decay)


def clipup(learning_rate: float, momentum: float = 0.9, max_speed: float = None) -> GradientTransformation:
    """ClipUp (Toklu et al. 2020), reference ``pgpe.py:29-59``."""
    max_speed = 2 * learning_rate if max_speed is None else max_speed

    def clip(x, limit):
        n = torch.linalg.norm(x)
        return torch.where(n > limit, x * (limit / n.clamp_min(1e-30)), x)

    def init(params):
        return (torch.zeros_like(params),)

    def update(grads, opt_state, params=None):
        (v,) = opt_state
        g = grads / torch.linalg.norm(grads).clamp_min(1e-30) * learning_rate
        v = clip(momentum * v + g, max_speed)
        return -v, (v,)

    return GradientTransformation(init, update)


_BY_NAME = {"sgd": sgd, "adam": adam, "adamw": adamw, "clipup": clipup}


def get_optimizer(name: str, **kwargs) -> GradientTransformation:
    if name not in _BY_NAME:
        raise ValueError(f"unknown optimizer {name}")
    return _BY_NAME[name](**kwargs)


class OptaxWrapper(Stateful):
    """An optimiser as a sub-module whose ``opt_state`` lives in the state tree."""

    def __init__(self, optimizer: GradientTransformation, init_params: torch.Tensor):
        super().__init__()
        self.optimizer = optimizer
        self.init_params = init_params

    def setup(self, key):
        return State(opt_state=self.optimizer.init(self.init_params))

    def update(self, state, grads, params=None):
        updates, opt_state = self.optimizer.update(grads, state.opt_state, params)
        return updates, state.update(opt_state=opt_state)


OptimizerWrapper = OptaxWrapper
