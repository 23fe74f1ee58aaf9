"""Decomposition containers (reference ``containers/clustered_algorithm.py:10-158``).

``ClusterdAlgorithm``: the dimensions are split into ``num_cluster`` equal blocks and
an independent copy of the base algorithm (own key) optimises each block; the full
population is the concatenation of the blocks and every copy receives the same
fitness.  ``RandomMaskAlgorithm`` updates only a random subset of ``num_cluster −
num_mask`` blocks, re-drawn every ``change_every`` generations (the reference's
version calls a removed API, ``clustered_algorithm.py:99``; this is the described
behaviour).
"""
from __future__ import annotations

import torch

from ...core import Algorithm, State, StackedModules, use_state
from ...ops import random as rnd


class ClusterdAlgorithm(Algorithm):
    def __init__(self, base_algorithm, dim, num_cluster):
        super().__init__()
        assert dim % num_cluster == 0
        self.dim, self.num_cluster = dim, num_cluster
        self.subproblem_dim = dim // num_cluster
        self.base_algorithms = StackedModules([base_algorithm] * num_cluster)
        self.pop_size = getattr(base_algorithm, "pop_size", None)

    def setup(self, key):
        return State()

    def ask(self, state):
        subs = []
        for k, alg in enumerate(self.base_algorithms):
            sub, state = use_state(alg.ask, k)(state)
            subs.append(sub)
        return torch.cat(subs, 1), state

    def tell(self, state, fitness):
        for k, alg in enumerate(self.base_algorithms):
            state = use_state(alg.tell, k)(state, fitness)
        return state


ClusteredAlgorithm = ClusterdAlgorithm


class RandomMaskAlgorithm(ClusterdAlgorithm):
    def __init__(self, base_algorithm, dim, num_cluster, num_mask=1, change_every=1, pop_size=None):
        super().__init__(base_algorithm, dim, num_cluster)
        assert 0 < num_mask < num_cluster
        self.num_mask, self.num_valid, self.change_every = num_mask, num_cluster - num_mask, change_every
        self.pop_size = pop_size if pop_size is not None else base_algorithm.pop_size

    def setup(self, key):
        return State(key=key, sub_pops=None, active=list(range(self.num_valid)), count=0)

    def init_ask(self, state):
        subs = []
        for k, alg in enumerate(self.base_algorithms):
            sub, state = use_state(alg.ask, k)(state)
            subs.append(sub)
        return torch.cat(subs, 1), state.update(sub_pops=subs)

    def ask(self, state):
        if state.count % self.change_every == 0:
            key, sub = rnd.split(state.key)
            active = sorted(rnd.permutation(sub, self.num_cluster)[: self.num_valid].tolist())
            state = state.update(key=key, active=active, count=0)
        subs = list(state.sub_pops)
        for k in state.active:
            subs[k], state = use_state(self.base_algorithms[k].ask, k)(state)
        return torch.cat(subs, 1), state.update(sub_pops=subs)

    def init_tell(self, state, fitness):
        for k, alg in enumerate(self.base_algorithms):
            state = use_state(alg.tell, k)(state, fitness)
        return state

    def tell(self, state, fitness):
        for k in state.active:
            state = use_state(self.base_algorithms[k].tell, k)(state, fitness)
        return state.update(count=state.count + 1)
