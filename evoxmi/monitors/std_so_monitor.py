"""Deprecated single-objective monitor (reference ``std_so_monitor.py:10-130``);
the fork's DE harness uses it (``run/run_de.py:67``)."""
from __future__ import annotations

import warnings

import torch

from ..core import Monitor


class StdSOMonitor(Monitor):
    def __init__(self, record_topk=1, record_fit_history=True, record_pop_history=False):
        super().__init__()
        warnings.warn("The StdSOMonitor is deprecated in favor of the new EvalMonitor.", DeprecationWarning)
        self.record_fit_history = record_fit_history
        self.record_pop_history = record_pop_history
        self.fitness_history = []
        self.population_history = []
        self.record_topk = record_topk
        self.current_population = None
        self.topk_solutions = None
        self.topk_fitness = None
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
        if self.record_fit_history:
            self.fitness_history.append(fitness.detach().clone())
        pop = self.current_population
        if pop is not None and pop.shape[0] != fitness.shape[0]:
            pop = None
        k = min(self.record_topk, fitness.shape[0])
        if k == 1:
            i = torch.argmin(fitness).reshape(1)
            fit = fitness.index_select(0, i)
            sol = pop.index_select(0, i) if pop is not None else None
            if self.topk_fitness is None:
                self.topk_fitness = fit.clone()
                self.topk_solutions = sol.clone() if sol is not None else None
            else:
                better = fit < self.topk_fitness
                self.topk_fitness = torch.where(better, fit, self.topk_fitness)
                if sol is not None and self.topk_solutions is not None:
                    self.topk_solutions = torch.where(better[:, None], sol, self.topk_solutions)
        else:
            f = fitness if self.topk_fitness is None else torch.cat([self.topk_fitness, fitness])
            s = pop
            if pop is not None and self.topk_solutions is not None:
                s = torch.cat([self.topk_solutions, pop], 0)
            v, i = torch.topk(f, k, largest=False, sorted=True)
            self.topk_fitness = v
            if s is not None and s.shape[0] == f.shape[0]:
                self.topk_solutions = s.index_select(0, i)

    def _d(self, x):
        od = self.opt_direction
        return x * (od.to(x.device) if isinstance(od, torch.Tensor) else od)

    def get_last(self):
        return self._d(self.fitness_history[-1])

    def get_topk_fitness(self):
        return self._d(self.topk_fitness)

    def get_topk_solutions(self):
        return self.topk_solutions

    def get_best_fitness(self):
        if self.topk_fitness is None:
            warnings.warn("trying to get info from a monitor with no recorded data")
            return None
        return self._d(self.topk_fitness[0])

    def get_best_solution(self):
        if self.topk_solutions is None:
            warnings.warn("trying to get info from a monitor with no recorded data")
            return None
        return self.topk_solutions[0]

    def get_history(self):
        return [self._d(f) for f in self.fitness_history]

    def flush(self):
        if torch.cuda.is_available() and torch.cuda.is_initialized():
            torch.cuda.synchronize()

    def close(self):
        self.flush()
