"""Independent runs of one algorithm as ONE batched computation.

The fork's benchmark protocol runs every DE variant 32 times per CEC'22 function
(reference ``run/run_de.py:54-114``): at D = 20 and pop = 100 a generation is a few
hundred tiny kernels, so one run at a time leaves the GPU idle between launches.
``BatchedRuns(algorithm, n_runs)`` keeps the n_runs states stacked along a leading
axis and executes ``ask``/``tell`` once for all of them with ``torch.func.vmap`` —
the reference's own mechanism for independent copies (``jax.vmap``) — so a launch
sequence advances every run.  The evaluation sees one (n_runs·pop, d) matrix.

Run ``r`` starts from ``split(key, n_runs)[r]`` and is bit-identical to running the
algorithm alone from that key (``tests/test_batched_runs.py``).  The HIP ops used by the
DE zoo (Philox streams, the fused trial kernel, sorts) carry vmap rules that fold the run
axis into their launch (``evoxmi/ops/batching.py``), so a batched generation costs the
same number of launches as a single run.
"""
from __future__ import annotations

import torch
from torch.func import vmap

from ...core import Algorithm, State
from ...ops import random as rnd


class BatchedRuns(Algorithm):
    def __init__(self, algorithm: Algorithm, n_runs: int):
        super().__init__()
        self._base = algorithm  # underscore: not a child module (its states live in `runs`)
        self.n_runs = int(n_runs)
        self.pop_size = getattr(algorithm, "pop_size", None)
        from ...ops import batching

        batching.register()  # vmap rules of the HIP ops (no-op cost after the first call)

    def wraps_init_ask(self):
        from ...core.algorithm import algorithm_has_init_ask

        return algorithm_has_init_ask(self._base)

    def run_keys(self, key):
        return rnd.split(key, self.n_runs)

    def setup(self, key):
        keys = self.run_keys(key)
        runs = vmap(self._base.init)(keys)
        return State(runs=runs)

    def _flat(self, pop):
        return pop.reshape((-1,) + tuple(pop.shape[2:]))

    def init_ask(self, state):
        if not self.wraps_init_ask():
            return None, state
        pop, runs = vmap(self._base.init_ask)(state.runs)
        return self._flat(pop), state.update(runs=runs)

    def init_tell(self, state, fitness):
        f = fitness.reshape((self.n_runs, -1) + tuple(fitness.shape[1:]))
        return state.update(runs=vmap(self._base.init_tell)(state.runs, f))

    def ask(self, state):
        pop, runs = vmap(self._base.ask)(state.runs)
        return self._flat(pop), state.update(runs=runs)

    def tell(self, state, fitness):
        f = fitness.reshape((self.n_runs, -1) + tuple(fitness.shape[1:]))
        return state.update(runs=vmap(self._base.tell)(state.runs, f))

    # ---------------------------------------------------------------- harness helpers
    def set_field(self, state, **fields):
        """Write a (scalar or per-run) value into every run's state, e.g. the fork's
        wall-clock ``progress`` injection (reference run/run_de.py:90-94)."""
        runs = state.runs
        upd = {}
        for k, v in fields.items():
            old = runs[k]
            v = torch.as_tensor(v, dtype=old.dtype, device=old.device) if not isinstance(v, torch.Tensor) else v.to(old.device, old.dtype)
            upd[k] = v.expand_as(old).clone() if v.shape != old.shape else v
        return state.update(runs=runs.update(**upd))

    def best_fitness(self, state):
        """Best fitness of every run, (n_runs,)."""
        return state.runs.fitness.reshape(self.n_runs, -1).min(1).values
