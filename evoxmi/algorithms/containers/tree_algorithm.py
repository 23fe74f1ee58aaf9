"""One base algorithm per leaf of a parameter pytree (reference ``containers/tree_algorithm.py:9-45``)."""
from __future__ import annotations

import torch
import torch.utils._pytree as pytree

from ...core import Algorithm, State, StackedModules, use_state


class FlattenParam:
    def __init__(self, dummy_input):
        self.shape_def = pytree.tree_map(lambda x: tuple(x.shape), dummy_input)

    def flatten(self, x):
        return pytree.tree_map(lambda v: v.reshape(v.shape[0], -1), x)

    def unflatten(self, x):
        leaves, spec = pytree.tree_flatten(x)
        shapes = pytree.tree_leaves(self.shape_def, is_leaf=lambda s: isinstance(s, tuple))
        return pytree.tree_unflatten([v.reshape(-1, *s) for v, s in zip(leaves, shapes)], spec)


class TreeAlgorithm(Algorithm):
    """``base_algorithm(*leaf_args)`` is built for every leaf of ``initial_params``
    (e.g. per-layer CMA-ES); the candidate pytree is the per-leaf populations reshaped
    to the leaf shapes."""

    def __init__(self, base_algorithm, initial_params, *args):
        super().__init__()
        self.flatten_param = FlattenParam(initial_params)
        built = pytree.tree_map(lambda *a: base_algorithm(*a), *args)
        self.inner, self.treedef = pytree.tree_flatten(built, is_leaf=lambda x: isinstance(x, Algorithm))
        for i, m in enumerate(self.inner):
            setattr(self, f"auto_gen_{i}", m)

    def setup(self, key):
        return State()

    def ask(self, state):
        params = []
        for m in self.inner:
            p, state = use_state(m.ask)(state)
            params.append(p)
        return self.flatten_param.unflatten(pytree.tree_unflatten(params, self.treedef)), state

    def tell(self, state, fitness):
        for m in self.inner:
            state = use_state(m.tell)(state, fitness)
        return state
