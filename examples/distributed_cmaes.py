"""CMA-ES with the population sharded over ranks (one process per GPU over RCCL; gloo ranks
on a CPU-only host).  Each rank samples only its own rows (Philox counters are global row
indices, so 1, 2, 4 or 8 ranks draw the same population), evaluates them, and the ranks
exchange the fitness and the partial covariance statistics; the decomposition is replicated.

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 examples/distributed_cmaes.py
    python examples/distributed_cmaes.py --gpus 2 --device cpu        # spawns 2 gloo ranks itself

A checkpoint of the (replicated) state is written by rank 0 and can be resumed with any
number of ranks (``--resume``).
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--device", default="cuda", choices=["cuda", "cpu"])
    ap.add_argument("--dim", type=int, default=100)
    ap.add_argument("--pop", type=int, default=1000)
    ap.add_argument("--generations", type=int, default=30)
    ap.add_argument("--checkpoint", default=None)
    ap.add_argument("--resume", action="store_true")
    a = ap.parse_args()
    from evoxmi.parallel.launch import ensure_ranks

    ensure_ranks(a.gpus, device=a.device)  # spawns the ranks unless started by torchrun
    import torch.distributed as dist

    from evoxmi import random as rnd
    from evoxmi.algorithms import CMAES
    from evoxmi.core.checkpoint import load_state, save_state
    from evoxmi.monitors import EvalMonitor
    from evoxmi.parallel import init_distributed
    from evoxmi.problems.numerical import Sphere
    from evoxmi.workflows import StdWorkflow

    rank, world, device = init_distributed(backend="gloo" if a.device == "cpu" else None)
    center = torch.full((a.dim,), 3.0, device=device)
    monitor = EvalMonitor()
    wf = StdWorkflow(CMAES(center_init=center, init_stdev=1.0, pop_size=a.pop), Sphere(), monitors=[monitor],
                     graph=device.type == "cuda")
    state = wf.init(rnd.PRNGKey(7, device=device))
    if a.resume and a.checkpoint and os.path.exists(a.checkpoint):
        state = load_state(a.checkpoint, map_location=device)
    if world > 1:
        state = wf.enable_distributed(state)
    for _ in range(a.generations):
        state = wf.step(state)
    best = float(monitor.get_best_fitness())
    if a.checkpoint and rank == 0:
        save_state(state, a.checkpoint)
    if rank == 0:
        print(f"ranks {world}: best fitness {best:.4e} after {int(state.generation)} generations", flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
