"""Algorithm base class (reference ``src/evox/core/algorithm.py:10-90``).

``ask(state) -> (population, state)`` proposes candidates, ``tell(state, fitness)
-> state`` consumes their (minimisation-oriented) fitness.  ``init_ask`` /
``init_tell`` are optional: when overridden, the workflow uses them at
generation 0 (the first population may differ in size from later ones).
"""
import contextlib
from typing import Hashable, Optional, Tuple

import torch

from .module import Stateful
from .state import State


class Algorithm(Stateful):
    """Base class for all algorithms."""

    def init_ask(self, state: State) -> Tuple[torch.Tensor, State]:
        return None, State()

    def init_tell(self, state: State, fitness: torch.Tensor) -> State:
        return State()

    def ask(self, state: State) -> Tuple[torch.Tensor, State]:
        return torch.zeros(0), State()

    def tell(self, state: State, fitness: torch.Tensor) -> State:
        return State()

    # ---- step variants: a host-known choice of how a generation runs (no device read)
    def graph_variant(self, generation: int) -> Optional[Hashable]:
        """Key of the step variant for workflow generation ``generation`` (``None``: the one
        default).  A hipGraph-capturing workflow captures one graph per distinct key over the
        same state buffers and replays the matching one; eager steps run inside
        :meth:`graph_variant_context` too (e.g. CMA-ES's longer cold-start eigensolver
        schedule for its first generations)."""
        return None

    def graph_variant_context(self, variant: Hashable):
        """Context manager active while a step of ``variant`` is captured or run eagerly."""
        return contextlib.nullcontext()

    def graph_variant_set(self) -> Tuple[Hashable, ...]:
        """Every variant :meth:`graph_variant` may return, including ones chosen only on a
        run-time condition (``StdWorkflow.prepare_graphs`` captures them all up front)."""
        return ()

    def after_step(self, generation: int) -> None:
        """Called by the workflow once the step that produced ``generation`` is enqueued (host
        side, no device read): e.g. to record an event whose completion a later
        :meth:`graph_variant` call polls."""


def algorithm_has_init_ask(algorithm: Algorithm, state: State = None) -> bool:
    """True when ``algorithm`` overrides ``init_ask`` (reference ``utils/common.py:15-19``).

    The reference probes the method with ``eval_shape``; without a tracer we inspect
    the class hierarchy instead, which gives the same answer for every algorithm
    that follows the base-class contract (``init_ask`` returning ``None`` = absent).
    """
    wraps = getattr(algorithm, "wraps_init_ask", None)  # containers answer for the wrapped algorithm
    if wraps is not None:
        return bool(wraps())
    return type(algorithm).init_ask is not Algorithm.init_ask
