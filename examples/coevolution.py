"""Container algorithms (the reference's docs/source/guide/user/4-container.md): two CSO
sub-swarms co-evolving the two 20-D halves of a 40-D Ackley problem.  ``VectorizedCoevolution``
updates every sub-population each generation; ``Coevolution`` one at a time.

    python examples/coevolution.py [--sequential] [--device cpu|cuda]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from evoxmi import random as rnd  # noqa: E402
from evoxmi.algorithms import CSO, Coevolution, VectorizedCoevolution  # noqa: E402
from evoxmi.monitors import EvalMonitor  # noqa: E402
from evoxmi.problems.numerical import Ackley  # noqa: E402
from evoxmi.workflows import StdWorkflow  # noqa: E402


def run(device: str = "cpu", sequential: bool = False, generations: int = 200):
    dev = torch.device(device)
    base = [CSO(lb=torch.full((20,), -32.0, device=dev), ub=torch.full((20,), 32.0, device=dev), pop_size=100) for _ in range(2)]
    container = Coevolution if sequential else VectorizedCoevolution
    algorithm = container(base, dim=40, num_subpops=2, random_subpop=False)
    monitor = EvalMonitor()
    workflow = StdWorkflow(algorithm, Ackley(), monitors=[monitor])
    state = workflow.init(rnd.PRNGKey(42, device=dev))
    for _ in range(generations):
        state = workflow.step(state)
    return float(monitor.get_best_fitness())


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--device", default="cpu")
    ap.add_argument("--sequential", action="store_true")
    a = ap.parse_args()
    print(f"best fitness {run(a.device, a.sequential):.3e}")
