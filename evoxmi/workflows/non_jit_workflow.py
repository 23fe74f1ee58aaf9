"""Eager workflow (reference ``src/evox/workflows/non_jit_workflow.py:8-150``).

Identical hook sequence to :class:`StdWorkflow` but never captures a graph and
lets the problem return host data (numpy / Python lists), which is converted to
a float32 tensor on the algorithm's device.
"""
from __future__ import annotations

import warnings

import numpy as np
import torch

from ..core import State, Workflow, use_state
from ..core.algorithm import algorithm_has_init_ask
from ..utils.common import parse_opt_direction


class NonJitWorkflow(Workflow):
    def __init__(self, algorithm, problem, monitors=(), opt_direction="min", sol_transforms=(), fit_transforms=(), pop_transform=None, monitor=None):
        super().__init__()
        self.algorithm = algorithm
        self.problem = problem
        self.monitors = list(monitors)
        if monitor is not None:
            warnings.warn("`monitor` is deprecated", DeprecationWarning)
            self.monitors = [monitor]
        self.registered_hooks = {h: [] for h in ("pre_step", "pre_ask", "post_ask", "pre_eval", "post_eval", "pre_tell", "post_tell", "post_step")}
        for m in self.monitors:
            for h in m.hooks():
                self.registered_hooks[h].append(m)
        self.opt_direction = parse_opt_direction(opt_direction)
        for m in self.monitors:
            m.set_opt_direction(self.opt_direction)
        self.sol_transforms = list(sol_transforms) if pop_transform is None else [pop_transform]
        self.fit_transforms = list(fit_transforms)
        self._has_init_ask = algorithm_has_init_ask(algorithm)

    def setup(self, key):
        return State(generation=0)

    def step(self, state):
        for m in self.registered_hooks["pre_step"]:
            m.pre_step(state)
        for m in self.registered_hooks["pre_ask"]:
            m.pre_ask(state)
        is_init = self._has_init_ask and state.generation == 0
        ask = self.algorithm.init_ask if is_init else self.algorithm.ask
        tell = self.algorithm.init_tell if is_init else self.algorithm.tell
        cand_sol, state = use_state(ask)(state)
        for m in self.registered_hooks["post_ask"]:
            m.post_ask(state, cand_sol)
        transformed = cand_sol
        for t in self.sol_transforms:
            transformed = t(transformed)
        for m in self.registered_hooks["pre_eval"]:
            m.pre_eval(state, cand_sol, transformed)
        fitness, state = use_state(self.problem.evaluate)(state, transformed)
        if not isinstance(fitness, torch.Tensor):
            fitness = torch.as_tensor(np.asarray(fitness), dtype=torch.float32)
        fitness = fitness.to(device=cand_sol.device, dtype=torch.float32)
        od = self.opt_direction
        fitness = fitness * (od.to(fitness.device) if isinstance(od, torch.Tensor) else od)
        for m in self.registered_hooks["post_eval"]:
            m.post_eval(state, cand_sol, transformed, fitness)
        tfit = fitness
        for t in self.fit_transforms:
            tfit = t(tfit)
        for m in self.registered_hooks["pre_tell"]:
            m.pre_tell(state, cand_sol, transformed, fitness, tfit)
        state = use_state(tell)(state, tfit)
        for m in self.registered_hooks["post_tell"]:
            m.post_tell(state)
        state = state.update(generation=state.generation + 1)
        for m in self.registered_hooks["post_step"]:
            m.post_step(state)
        return state
