"""PSO on Ackley (d = 2), the reference's first example
(/root/reference/docs/source/example/pso_ackley.ipynb): population 100, bounds [-32, 32],
100 generations, key 42.  The reference prints best fitness 0.0 at x ≈ (-4.0e-7, 5.3e-7); at
the same x the f32 Ackley is one rounding step above zero, which is what this run reaches
(tests/test_examples.py pins best ≤ 1e-6 and |x|∞ ≤ 1e-6).

    python examples/pso_ackley.py [--device cpu|cuda]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from evoxmi import algorithms, monitors, problems, workflows  # noqa: E402
from evoxmi import random as rnd  # noqa: E402


def run(device: str = "cpu", generations: int = 100, seed: int = 42):
    dev = torch.device(device)
    algorithm = algorithms.PSO(lb=torch.full((2,), -32.0, device=dev), ub=torch.full((2,), 32.0, device=dev), pop_size=100)
    problem = problems.numerical.Ackley()
    monitor = monitors.EvalMonitor()
    workflow = workflows.StdWorkflow(algorithm, problem, monitors=[monitor])
    state = workflow.init(rnd.PRNGKey(seed, device=dev))
    for _ in range(generations):
        state = workflow.step(state)
    return float(monitor.get_best_fitness()), monitor.get_best_solution().cpu()


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--device", default="cpu")
    a = ap.parse_args()
    best, x = run(a.device)
    print(f"best fitness {best:.3e} at x = {x.tolist()}")
