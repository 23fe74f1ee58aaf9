"""Seed sensitivity of tests/test_eigh_sbr.py::test_cmaes_trajectories_sbr_vs_library_eigh: the
median-over-5-seeds progress ratio of CMA-ES (λ 10⁴, d 1000, Ellipsoid, 100 generations) with the
device SBR solver vs rocSOLVER, for several disjoint seed sets and both correction precisions.

    python tools/parity_probe.py [--sets 3]
"""
import argparse
import json
import math
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def traj(impl, seed, prec):
    from evoxmi import config as cfg
    from evoxmi import random as rnd
    from evoxmi.algorithms import CMAES
    from evoxmi.problems.numerical import Ellipsoid
    from evoxmi.workflows import StdWorkflow

    with cfg.override(eigh=impl, sbr_device_iters=16, sbr_corr_prec=prec):
        center = (torch.rand(1000, generator=torch.Generator().manual_seed(1)) * 10 - 5).cuda()
        algo = CMAES(center_init=center, init_stdev=1.0, pop_size=10000)
        prob = Ellipsoid()
        wf = StdWorkflow(algo, prob, graph=(impl == "sbr"))
        st = wf.init(rnd.PRNGKey(seed, device=torch.device("cuda")))
        pst = st.get_child_state("problem")
        f = []
        for _ in range(100):
            st = wf.step(st)
            a = st.get_child_state("algorithm")
            f.append(float(prob.evaluate(pst, a.mean.reshape(1, -1))[0][0]))
        return f


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sets", type=int, default=3)
    a = ap.parse_args()
    for k in range(a.sets):
        seeds = list(range(7 + 5 * k, 12 + 5 * k))
        torch_runs = [traj("torch", s, "x6") for s in seeds]
        med_t = [statistics.median(r[g] for r in torch_runs) for g in range(100)]
        prog_t = math.log(med_t[10] / med_t[99])
        out = {"seeds": seeds, "prog_torch": round(prog_t, 4)}
        for prec in ("x6", "x3"):
            runs = [traj("sbr", s, prec) for s in seeds]
            med = [statistics.median(r[g] for r in runs) for g in range(100)]
            prog = math.log(med[10] / med[99])
            logr = statistics.median(abs(math.log(med[g] / med_t[g])) for g in range(10, 100))
            out[prec] = {"prog": round(prog, 4), "prog_ratio_dev": round(prog / prog_t - 1, 4), "median_log_ratio": round(logr, 4),
                         "per_seed_prog": [round(math.log(r[10] / r[99]), 3) for r in runs]}
        out["per_seed_prog_torch"] = [round(math.log(r[10] / r[99]), 3) for r in torch_runs]
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
