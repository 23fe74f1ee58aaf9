"""Deprecated multi-objective monitor (reference ``std_mo_monitor.py:13-111``)."""
from __future__ import annotations

import warnings

import torch

from ..core import Monitor


class StdMOMonitor(Monitor):
    def __init__(self, record_pf=False, record_fit_history=True, record_pop_history=False):
        super().__init__()
        warnings.warn("The StdMOMonitor is deprecated in favor of the new EvalMonitor.", DeprecationWarning)
        self.record_pf = record_pf
        self.record_fit_history = record_fit_history
        self.record_pop_history = record_pop_history
        self.fitness_history = []
        self.population_history = []
        self.current_population = None
        self.pf_solutions = None
        self.pf_fitness = None
        self.opt_direction = 1

    def set_opt_direction(self, opt_direction):
        self.opt_direction = opt_direction

    def hooks(self):
        return ["post_ask", "post_eval"]

    def post_ask(self, _state, cand_sol):
        self.record_pop(cand_sol)

    def post_eval(self, _state, _cand_sol, _transformed, fitness):
        self.record_fit(fitness)

    def record_pop(self, pop, transform=None):
        if self.record_pop_history:
            self.population_history.append(pop.detach().clone())
        self.current_population = pop

    def record_fit(self, fitness, metrics=None, transform=None):
        from ..operators.selection.non_dominate import non_dominated_sort

        if self.record_fit_history:
            self.fitness_history.append(fitness.detach().clone())
        if self.record_pf:
            f = fitness if self.pf_fitness is None else torch.cat([self.pf_fitness, fitness], 0)
            s = self.current_population if self.pf_solutions is None else torch.cat([self.pf_solutions, self.current_population], 0)
            keep = non_dominated_sort(f) == 0
            self.pf_fitness, self.pf_solutions = f[keep], s[keep]

    def _d(self, x):
        od = self.opt_direction
        return x * (od.to(x.device) if isinstance(od, torch.Tensor) else od)

    def get_last(self):
        return self._d(self.fitness_history[-1])

    def get_pf_fitness(self):
        return self._d(self.pf_fitness)

    def get_pf_solutions(self):
        return self.pf_solutions

    def get_history(self):
        return [self._d(f) for f in self.fitness_history]

    def flush(self):
        if torch.cuda.is_available() and torch.cuda.is_initialized():
            torch.cuda.synchronize()

    def close(self):
        self.flush()
