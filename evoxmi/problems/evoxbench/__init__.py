"""EvoXBench NAS benchmark problems (reference ``problems/evoxbench/evoxbench.py:13-75``).

The benchmark is a host-side package with a database download; it is not part of
this image, so the classes import lazily and raise a clear error when the package
is absent.  With ``evoxbench`` installed they evaluate the (host) benchmark with a
seed drawn from the problem key, exactly like the reference's ``io_callback``.
"""
from __future__ import annotations

import numpy as np
import torch

from ...core import Problem, State
from ...ops import random as rnd


def _bench(kind, pid):
    try:
        from evoxbench.test_suites import c10mop, citysegmop, in1kmop  # type: ignore
    except ImportError as e:
        raise ImportError("EvoXBench problems need the `evoxbench` package and its database (not available here)") from e
    return {"c10mop": c10mop, "citysegmop": citysegmop, "in1kmop": in1kmop}[kind](pid)


class EvoXBenchProblem(Problem):
    def __init__(self, benchmark):
        super().__init__()
        self.benchmark = benchmark
        self.n_objs = benchmark.evaluator.n_objs
        self.lb = torch.as_tensor(benchmark.search_space.lb)
        self.ub = torch.as_tensor(benchmark.search_space.ub)

    def setup(self, key):
        return State(key=key)

    def evaluate(self, state, pop):
        key, sub = rnd.split(state.key)
        seed = int(rnd.randint(sub, (1,), 0, 2**31 - 1)[0])
        np.random.seed(seed)
        fit = self.benchmark.evaluate(pop.detach().cpu().numpy()).astype(np.float32)
        return torch.as_tensor(fit, device=pop.device), state.update(key=key)


class C10MOP(EvoXBenchProblem):
    def __init__(self, problem_id):
        assert isinstance(problem_id, int) and 1 <= problem_id <= 9, "For c10mop, problem_id must be an integer between 1 and 9"
        super().__init__(_bench("c10mop", problem_id))


class CitySegMOP(EvoXBenchProblem):
    def __init__(self, problem_id):
        assert isinstance(problem_id, int) and 1 <= problem_id <= 15, "For citysegmop, problem_id must be an integer between 1 and 15"
        super().__init__(_bench("citysegmop", problem_id))


class IN1kMOP(EvoXBenchProblem):
    def __init__(self, problem_id):
        assert isinstance(problem_id, int) and 1 <= problem_id <= 9, "For in1kmop, problem_id must be an integer between 1 and 9"
        super().__init__(_bench("in1kmop", problem_id))
