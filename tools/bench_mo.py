"""Multi-objective north-star throughput (BASELINE.json configs 3 and 5).

  nsga2 : NSGA-II pop=4096 on DTLZ2 (m=3, d=500)           — 1×MI355X
  moead : MOEA/D pop=16384 on LSMOP1 (m=3, d=10000), Tchebycheff aggregation

python tools/bench_mo.py --algo nsga2|moead [--gens 20] [--warmup 3] [--no-graph]

Prints one JSON line: generations/s and evaluations/s of full generations
(ask → evaluate → tell), random-init populations, fp32.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def build(args, dev):
    from evoxmi.algorithms import MOEAD, NSGA2
    from evoxmi.problems.numerical import DTLZ2, LSMOP1

    m = 3
    if args.algo == "nsga2":
        d = args.dim or 500
        lb, ub = torch.zeros(d, device=dev), torch.ones(d, device=dev)
        return NSGA2(lb, ub, m, args.pop or 4096), DTLZ2(d=d, m=m)
    d = args.dim or 10000
    lb = torch.zeros(d, device=dev)
    ub = torch.cat([torch.ones(m - 1, device=dev), 10 * torch.ones(d - m + 1, device=dev)])
    return MOEAD(lb, ub, m, args.pop or 16384, func_name="tchebycheff"), LSMOP1(d=d, m=m)


def main():
    from evoxmi import random as rnd
    from evoxmi.workflows import StdWorkflow

    ap = argparse.ArgumentParser()
    ap.add_argument("--algo", choices=["nsga2", "moead"], default="nsga2")
    ap.add_argument("--pop", type=int, default=0)
    ap.add_argument("--dim", type=int, default=0)
    ap.add_argument("--gens", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--cpu", action="store_true")
    args = ap.parse_args()
    dev = torch.device("cpu" if args.cpu else "cuda")
    algo, prob = build(args, dev)

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize()

    wf = StdWorkflow(algo, prob, graph=not (args.no_graph or args.cpu))
    st = wf.init(rnd.PRNGKey(7, device=dev))
    for _ in range(1 + args.warmup):
        st = wf.step(st)
    sync()
    t = time.perf_counter()
    for _ in range(args.gens):
        st = wf.step(st)
    sync()
    dt = (time.perf_counter() - t) / args.gens
    fit = st.get_child_state("algorithm").fitness
    pop = algo.pop_size
    print(json.dumps({
        "config": args.algo, "pop": pop, "dim": algo.dim, "n_objs": 3, "graph": not (args.no_graph or args.cpu),
        "ms_per_gen": round(dt * 1e3, 3), "gens_per_sec": round(1 / dt, 2), "evals_per_sec": round(pop / dt, 1),
        "fitness_finite": bool(torch.isfinite(fit).all()), "mean_obj": [round(float(v), 4) for v in fit.mean(0)],
    }))


if __name__ == "__main__":
    main()
