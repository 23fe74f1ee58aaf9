"""OpenES + Brax-style Ant throughput (north-star config 4 shape: pop 8192, MLP 27-64-64-8).

python tools/bench_neuro.py [--pop 8192] [--cap 1000] [--gens 5]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    from evoxmi import random as rnd
    from evoxmi.algorithms import OpenES
    from evoxmi.models import MLPPolicy
    from evoxmi.problems.neuroevolution import Brax
    from evoxmi.utils import TreeAndVector, rank_based_fitness
    from evoxmi.workflows import StdWorkflow

    ap = argparse.ArgumentParser()
    ap.add_argument("--pop", type=int, default=8192)
    ap.add_argument("--cap", type=int, default=1000)
    ap.add_argument("--gens", type=int, default=5)
    ap.add_argument("--hidden", type=int, default=64)
    args = ap.parse_args()
    dev = torch.device("cuda")
    policy = MLPPolicy([27, args.hidden, args.hidden, 8])
    params = policy.init(rnd.PRNGKey(0), device=dev)
    tv = TreeAndVector(params)
    algo = OpenES(tv.to_vector(params), args.pop, learning_rate=0.01, noise_stdev=0.05, optimizer="adam")
    wf = StdWorkflow(algo, Brax(policy, "ant", args.cap), sol_transforms=[tv.batched_to_tree], fit_transforms=[rank_based_fitness],
                     opt_direction="max")
    st = wf.init(rnd.PRNGKey(1, device=dev))
    st = wf.step(st)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(args.gens):
        st = wf.step(st)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / args.gens
    out = {"pop": args.pop, "cap_episode": args.cap, "params": policy.num_params, "ms_per_gen": round(dt * 1e3, 2),
           "gens_per_sec": round(1 / dt, 3), "env_steps_per_sec": round(args.pop * args.cap / dt, 1)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
