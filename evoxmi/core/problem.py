"""Problem base class (reference ``src/evox/core/problem.py:9-31``)."""
from typing import Any, Tuple

import torch

from .module import Stateful
from .state import State


class Problem(Stateful):
    """``evaluate(state, pop) -> (fitness, state)``; fitness is (N,) or (N, m)."""

    def evaluate(self, state: State, pop: Any) -> Tuple[torch.Tensor, State]:
        return torch.empty(0), state

    def valid(self, state: State, metric: str = "loss") -> State:
        """Switch the problem to validation mode (optional)."""
        return state
