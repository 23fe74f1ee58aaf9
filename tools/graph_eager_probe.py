"""Where do graph-mode and eager CMA-ES (d 64, λ 256) diverge?  Prints per generation the
mean checksum, eigen stats and the solver's plan for both modes."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from evoxmi import random as rnd  # noqa: E402
from evoxmi.algorithms import CMAES  # noqa: E402
from evoxmi.ops import eigh as E  # noqa: E402
from evoxmi.problems.numerical import F1_CEC2022  # noqa: E402
from evoxmi.workflows import StdWorkflow  # noqa: E402

d = int(sys.argv[1]) if len(sys.argv) > 1 else 64
for graph in (False, True):
    alg = CMAES(torch.zeros(d, device="cuda"), init_stdev=10.0, pop_size=256)
    wf = StdWorkflow(alg, F1_CEC2022(), graph=graph)
    st = wf.init(rnd.PRNGKey(7, device="cuda"))
    E.HISTORY.clear()
    for g in range(6):
        st = wf.step(st)
        a = st.get_child_state("algorithm")
        torch.cuda.synchronize()
        print(graph, g, f"mean {float(a.mean.double().sum()):.6f} sigma {float(a.sigma):.6f} C {float(a.C.double().sum()):.6f} B {float(a.B.double().abs().sum()):.6f}",
              [(h.refine_iters, round(h.off_rel, 9)) for h in list(E.HISTORY)[-2:]], list(alg._eig_plans.values()), flush=True)
