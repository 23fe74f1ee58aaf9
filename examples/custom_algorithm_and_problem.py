"""A custom Algorithm and Problem (the reference's
/root/reference/docs/source/example/custom_algorithm_and_problem.ipynb): a bit-flip + one-point
GA on one-max, maximised through ``opt_direction="max"``.

Everything an algorithm carries between generations lives in its ``State`` (returned by
``setup`` and updated immutably by ``ask`` / ``tell``), so the same class runs eagerly, inside a
hipGraph-captured generation on a GPU, or sharded across ranks.

    python examples/custom_algorithm_and_problem.py [--device cpu|cuda]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from evoxmi import Algorithm, Problem, State, monitors, workflows  # noqa: E402
from evoxmi import random as rnd  # noqa: E402
from evoxmi.operators import crossover, mutation  # noqa: E402


class OneMax(Problem):
    def evaluate(self, state, bitstrings):
        # (pop, bits) → number of ones per row
        return bitstrings.to(torch.float32).sum(dim=1), state


class CustomGA(Algorithm):
    def __init__(self, pop_size: int, ndim: int, flip_prob: float):
        super().__init__()
        self.pop_size, self.ndim, self.flip_prob = pop_size, ndim, flip_prob

    def setup(self, key):
        key, sub = rnd.split(key)
        pop = rnd.uniform(sub, (self.pop_size, self.ndim)) < 0.5
        return State(pop=pop, offsprings=torch.zeros((2 * self.pop_size, self.ndim), dtype=torch.bool, device=pop.device),
                     fit=torch.full((self.pop_size,), float("inf"), device=pop.device), key=key)

    def ask(self, state):
        key, mut_key, x_key = rnd.split(state.key, 3)
        # no mating selection: the offspring is twice the population
        offsprings = torch.cat([mutation.bitflip(mut_key, state.pop, self.flip_prob), crossover.one_point(x_key, state.pop)], dim=0)
        return offsprings, state.update(offsprings=offsprings, key=key)

    def tell(self, state, fitness):
        # the workflow hands minimisation fitness (−ones for opt_direction="max"): keep the best
        merged_pop = torch.cat([state.pop, state.offsprings], dim=0)
        merged_fit = torch.cat([state.fit, fitness], dim=0)
        idx = torch.argsort(merged_fit)[: self.pop_size]
        return state.update(pop=merged_pop[idx], fit=merged_fit[idx])


def run(device: str = "cpu", generations: int = 40, seed: int = 42):
    dev = torch.device(device)
    algorithm = CustomGA(pop_size=128, ndim=100, flip_prob=0.1)
    monitor = monitors.EvalMonitor()
    workflow = workflows.StdWorkflow(algorithm, OneMax(), monitors=[monitor], opt_direction="max")
    state = workflow.init(rnd.PRNGKey(seed, device=dev))
    trace = []
    for _ in range(generations):
        state = workflow.step(state)
        trace.append(float(monitor.get_best_fitness()))
    return trace, monitor.get_best_solution()


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--device", default="cpu")
    a = ap.parse_args()
    trace, sol = run(a.device)
    print(f"best ones after 20 / 40 generations: {trace[19]:.0f} / {trace[-1]:.0f} of 100")
