"""Population monitor (reference ``src/evox/monitors/pop_monitor.py:13-106``)."""
from __future__ import annotations

import warnings

import torch

from ..core import Monitor


class PopMonitor(Monitor):
    def __init__(self, population_name="population", fitness_name="fitness", fitness_only=False, to_host=False):
        super().__init__()
        self.population_name = population_name
        self.fitness_name = fitness_name
        self.fitness_only = fitness_only
        self.to_host = to_host
        self.population_history = []
        self.fitness_history = []

    def hooks(self):
        return ["post_step"]

    def _keep(self, x):
        x = x.detach()
        return x.to("cpu", non_blocking=True) if self.to_host else x.clone()

    def post_step(self, state):
        alg = state.get_child_state("algorithm")
        if not self.fitness_only:
            self.population_history.append(self._keep(getattr(alg, self.population_name)))
        self.fitness_history.append(self._keep(getattr(alg, self.fitness_name)))

    def get_latest_fitness(self):
        return self.fitness_history[-1]

    def get_latest_population(self):
        return self.population_history[-1]

    def get_population_history(self):
        return self.population_history

    def get_fitness_history(self):
        return self.fitness_history

    def plot(self, problem_pf=None, **kwargs):
        from ..vis_tools import plot

        if not self.fitness_history:
            warnings.warn("No fitness history recorded, return None")
            return None
        fh = [f.cpu() for f in self.fitness_history]
        if fh[0].ndim == 1:
            return plot.plot_obj_space_1d(fh, **kwargs)
        m = fh[0].shape[1]
        if m == 2:
            return plot.plot_obj_space_2d(fh, problem_pf, **kwargs)
        if m == 3:
            return plot.plot_obj_space_3d(fh, problem_pf, **kwargs)
        warnings.warn("Not supported yet.")
        return None

    def flush(self):
        if torch.cuda.is_available() and torch.cuda.is_initialized():
            torch.cuda.synchronize()
