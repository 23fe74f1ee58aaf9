"""PGPE with ClipUp (Sehnke et al. 2010, Toklu et al. 2020; reference ``es_variants/pgpe.py:29-130``).

Symmetric sampling ``c ± ε·σ``; the centre follows ``Δx = mean((f⁺ − f⁻)/2 · ε)``
through an optimiser sub-module (``'clipup'``, any optimiser name of
:mod:`evoxmi.utils.optim`, a GradientTransformation or a Stateful), the per-dimension
stdev follows ``mean(((f⁺+f⁻)/2 − f̄)(ε² − σ²)/σ)`` clipped to ±max_change·σ.
"""
from __future__ import annotations

import torch

from ....core import Algorithm, State, Stateful, use_state
from ....ops import random as rnd
from ....utils import optim
from ....parallel.dim_sharded import ColumnSeparable


def _l2(x):
    return torch.sqrt((x * x).sum())


class ClipUp(Stateful):
    """ClipUp as a Stateful (reference ``pgpe.py:29-59``): normalised gradient step with
    momentum and a maximum speed; returns the update ``−v``."""

    def __init__(self, step_size, max_speed, momentum, params):
        super().__init__()
        self.step_size, self.max_speed, self.momentum, self.params = step_size, max_speed, momentum, params

    def setup(self, key):
        return State(velocity=torch.zeros_like(self.params))

    _col_sum = None  # set under decision-axis sharding: the norms sum squares over every rank's columns

    def _norm(self, x):
        sq = (x * x).sum()
        return torch.sqrt(self._col_sum(sq) if self._col_sum is not None else sq)

    def update(self, state, gradient, _params=None):
        velocity = self.momentum * state.velocity + self.step_size * gradient / self._norm(gradient)
        vn = self._norm(velocity)
        velocity = torch.where(vn > self.max_speed, self.max_speed * velocity / vn, velocity)
        return -velocity, state.update(velocity=velocity)


class PGPE(ColumnSeparable, Algorithm):
    # decision-axis state sharding (P2): centre, stdev and noise are column blocks (noise drawn
    # per global column), the optimiser's state too; ClipUp's two norms all-reduce their sums
    # of squares (col_sum)
    column_separable = True
    dim_fields = ("center", "stdev", "noise")

    def __init__(self, pop_size, center_init, optimizer, stdev_init=0.1, center_learning_rate=0.15, stdev_learning_rate=0.1,
                 stdev_max_change=0.2):
        super().__init__()
        self.pop_size = pop_size
        self.center_init = center_init
        self.stdev_init = stdev_init
        self.center_learning_rate = center_learning_rate
        self.stdev_learning_rate = stdev_learning_rate
        self.stdev_max_change = stdev_max_change
        self.dim = center_init.shape[0]
        if isinstance(optimizer, str):
            if optimizer == "clipup":
                optimizer = ClipUp(step_size=0.15, max_speed=0.3, momentum=0.9, params=center_init)
            elif optimizer in optim._BY_NAME:
                optimizer = optim.OptaxWrapper(optim.get_optimizer(optimizer, learning_rate=center_learning_rate), center_init)
            else:
                raise ValueError(f"Unknown optimizer {optimizer}")
        elif isinstance(optimizer, optim.GradientTransformation):
            optimizer = optim.OptaxWrapper(optimizer, center_init)
        elif not isinstance(optimizer, Stateful):
            raise TypeError(f"{optimizer} is not supported right now")
        self.optimizer = optimizer

    def dim_shard(self, state, col0: int, own: int):
        if isinstance(self.optimizer, ClipUp):
            self.dim_child_fields = {"optimizer": ("velocity",)}
            self.optimizer._col_sum = self.col_sum
        elif isinstance(self.optimizer, optim.OptaxWrapper):
            self.dim_child_fields = {"optimizer": ("opt_state",)}
        else:
            raise ValueError("PGPE column sharding needs ClipUp or an element-wise optax-style optimiser")
        return super().dim_shard(state, col0, own)

    def setup(self, key):
        dev = self.center_init.device
        return State(center=self.center_init.clone(), stdev=torch.full((self.dim,), float(self.stdev_init), device=dev), key=key,
                     noise=torch.zeros((self.pop_size // 2, self.dim), device=dev))

    def ask(self, state):
        key, sub = rnd.split(state.key)
        noise = self.normal_cols(sub, self.pop_size // 2, state.center.device) * state.stdev
        return torch.cat([state.center + noise, state.center - noise], 0), state.update(key=key, noise=noise)

    def tell(self, state, fitness):
        h = self.pop_size // 2
        F_pos, F_neg = fitness[:h], fitness[h:]
        delta_x = (((F_pos - F_neg) / 2)[:, None] * state.noise).mean(0)
        f_avg = fitness.mean()
        delta_stdev = (((F_pos + F_neg) / 2 - f_avg)[:, None] * ((state.noise**2 - state.stdev**2) / state.stdev)).mean(0)
        updates, state = use_state(self.optimizer.update)(state, delta_x, state.center)
        center = state.center + updates
        bound = torch.abs(state.stdev * self.stdev_max_change)
        stdev_updates = torch.maximum(torch.minimum(self.stdev_learning_rate * delta_stdev, bound), -bound)
        return state.update(center=center, stdev=state.stdev - stdev_updates)
