"""Best-fitness trajectories of CMA-ES (λ = 10⁴, d = 1000, CEC'22 F1, 100 generations) with
the SBR eigensolver and with the library eigh, for several seeds (seed-to-seed spread vs
solver-to-solver difference; tests/test_eigh_sbr.py pins the comparison)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from evoxmi import config as cfg  # noqa: E402
from evoxmi import random as rnd  # noqa: E402
from evoxmi.algorithms import CMAES  # noqa: E402
from evoxmi.monitors import EvalMonitor  # noqa: E402
from evoxmi.problems.numerical import CEC2022TestSuit  # noqa: E402
from evoxmi.workflows import StdWorkflow  # noqa: E402


def traj(impl, seed, gens=100, problem="f1"):
    from evoxmi.problems.numerical import Ellipsoid

    with cfg.override(eigh=impl):
        if problem == "f1":
            center = (torch.rand(1000, generator=torch.Generator().manual_seed(1)) * 160 - 80).cuda()
            algo = CMAES(center_init=center, init_stdev=20.0, pop_size=10000)
            prob = CEC2022TestSuit.create(1)
        else:
            center = (torch.rand(1000, generator=torch.Generator().manual_seed(1)) * 10 - 5).cuda()
            algo = CMAES(center_init=center, init_stdev=1.0, pop_size=10000)
            prob = Ellipsoid()
        mon = EvalMonitor()
        wf = StdWorkflow(algo, prob, monitors=[mon], graph=(impl == "sbr"))
        st = wf.init(rnd.PRNGKey(seed, device=torch.device("cuda")))
        out = []
        pst = st.get_child_state("problem")
        for _ in range(gens):
            st = wf.step(st)
            # fitness at the distribution mean: the algorithm's progress (best-so-far is
            # dominated by lucky early samples while σ adapts)
            m = st.get_child_state("algorithm").mean.reshape(1, -1)
            out.append(float(prob.evaluate(pst, m)[0][0]))
        return out


if __name__ == "__main__":
    seeds = [int(s) for s in (sys.argv[1] if len(sys.argv) > 1 else "7,8,9").split(",")]
    problem = sys.argv[2] if len(sys.argv) > 2 else "f1"
    res = {impl: {s: traj(impl, s, problem=problem) for s in seeds} for impl in ("sbr", "torch")}
    for impl in res:
        for s in seeds:
            t = res[impl][s]
            print(impl, s, [f"{t[g]:.4g}" for g in (0, 5, 10, 20, 40, 60, 80, 99)], flush=True)
    json.dump(res, open(os.path.join(os.environ.get("GRAFT_REPO_ROOT", "."), "gpurun_out", "traj_probe.json"), "w"))
