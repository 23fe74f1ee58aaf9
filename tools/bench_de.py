"""Generations/s of every DE variant on CEC'22 (graph vs eager), the fork's workload shape.

python tools/bench_de.py [--dim 20] [--pop 100] [--gens 300] [--algos LSHADE,JSO]
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
    from evoxmi.algorithms import de_variants
    from evoxmi.problems.numerical import CEC2022TestSuit
    from evoxmi.workflows import StdWorkflow

    ap = argparse.ArgumentParser()
    ap.add_argument("--dim", type=int, default=20)
    ap.add_argument("--pop", type=int, default=100)
    ap.add_argument("--gens", type=int, default=300)
    ap.add_argument("--func", type=int, default=1)
    ap.add_argument("--algos", default=",".join(de_variants.__all__))
    args = ap.parse_args()
    dev = torch.device("cuda")
    D = args.dim
    lb, ub = torch.full((D,), -100.0, device=dev), torch.full((D,), 100.0, device=dev)
    out = {}
    for name in args.algos.split(","):
        row = {}
        for graph in (False, True):
            algo = getattr(de_variants, name)(lb=lb, ub=ub, pop_size=args.pop)
            wf = StdWorkflow(algo, CEC2022TestSuit.create(args.func), graph=graph)
            st = wf.init(rnd.PRNGKey(0, device=dev))
            for _ in range(5):
                st = wf.step(st)
            torch.cuda.synchronize()
            t = time.perf_counter()
            for i in range(args.gens):
                st = wf.step(st)
                a = st.get_child_state("algorithm")
                if "progress" in a.keys():
                    st = st.update_child("algorithm", a.update(progress=i / args.gens))
            torch.cuda.synchronize()
            dt = time.perf_counter() - t
            row["graph" if graph else "eager"] = round(args.gens / dt, 1)
        best = float(st.get_child_state("algorithm").fitness.min())
        row["best_f"] = best
        out[name] = row
        from evoxmi.ops.evo import kernel_error_flags
        row["kernel_err"] = kernel_error_flags()
        print(name, row, flush=True)
    print(json.dumps({"dim": D, "pop": args.pop, "func": args.func, "gens_per_sec": out}))


if __name__ == "__main__":
    main()
