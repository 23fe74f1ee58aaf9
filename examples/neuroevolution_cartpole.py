"""Neuroevolution on the batched on-device CartPole (the reference's gym_classic_control
example, with the environment stepped as tensors instead of gym worker processes): a
4-16-2 MLP policy, its weights flattened for the optimiser by ``TreeAndVector``, evolved with
PSO to maximise the episode return.  On a GPU the rollout runs inside the generation's
hipGraph.

    python examples/neuroevolution_cartpole.py [--device cpu|cuda] [--generations 20]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from evoxmi import random as rnd  # noqa: E402
from evoxmi.algorithms import PSO  # noqa: E402
from evoxmi.models import MLPPolicy  # noqa: E402
from evoxmi.monitors import EvalMonitor  # noqa: E402
from evoxmi.problems.neuroevolution.reinforcement_learning import Brax  # noqa: E402
from evoxmi.utils import TreeAndVector  # noqa: E402
from evoxmi.workflows import StdWorkflow  # noqa: E402


def run(device: str = "cpu", generations: int = 20, pop: int = 64, cap: int = 200):
    dev = torch.device(device)
    policy = MLPPolicy([4, 16, 2], activation="tanh", output_activation=None)
    params = policy.init(rnd.PRNGKey(0, device=dev))
    adapter = TreeAndVector(params)
    center = adapter.to_vector(params)
    algorithm = PSO(lb=torch.full_like(center, -5.0), ub=torch.full_like(center, 5.0), pop_size=pop)
    problem = Brax(policy, "cartpole", cap_episode=cap)
    monitor = EvalMonitor()
    workflow = StdWorkflow(algorithm, problem, monitors=[monitor], sol_transforms=[adapter.batched_to_tree], opt_direction="max")
    state = workflow.init(rnd.PRNGKey(42, device=dev))
    best = []
    for _ in range(generations):
        state = workflow.step(state)
        best.append(float(monitor.get_best_fitness()))
    return best


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--device", default="cpu")
    ap.add_argument("--generations", type=int, default=20)
    a = ap.parse_args()
    best = run(a.device, a.generations)
    print(f"best episode return: {best[0]:.0f} after 1 generation, {best[-1]:.0f} after {len(best)}")
