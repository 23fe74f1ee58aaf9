"""Convergence probe of the warm-started Jacobi eigensolver along a CMA-ES run
(bench config: pop 10 000, d 1000, CEC'22 F1).  For selected generations the same
(C, B_prev) is decomposed with 1, 2 and 3 sweeps; prints the relative off-diagonal
norm and the eigen-residual ‖C B − B diag(w)‖_F / ‖C‖_F of each, plus the time."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("EVOXMI_CMA_FUSED", "0")  # the probe hooks warm_eigh (the unfused epilogue's entry point)
import torch  # noqa: E402

from evoxmi import random as rnd  # noqa: E402
from evoxmi.algorithms import CMAES  # noqa: E402
from evoxmi.ops import jacobi  # noqa: E402
from evoxmi.problems.numerical import CEC2022TestSuit  # noqa: E402
from evoxmi.workflows import StdWorkflow  # noqa: E402

dev = torch.device("cuda")
gens = int(sys.argv[1]) if len(sys.argv) > 1 else 60
orig = jacobi.warm_eigh
log = []


def probe(C, B_prev=None, max_sweeps=None, tol=None, return_stats=False):
    g = len(log)
    if B_prev is not None and g % 10 == 0:
        rec = {"gen": g}
        for sw in (1, 2, 3):
            torch.cuda.synchronize()
            t = time.perf_counter()
            w, B, st = orig(C.clone(), B_prev.clone(), max_sweeps=sw, tol=1e-12, return_stats=True)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t
            res = torch.linalg.norm(C @ B - B * w) / torch.linalg.norm(C)
            orth = torch.linalg.norm(B.T @ B - torch.eye(B.shape[0], device=dev))
            rec[f"s{sw}"] = {"off_rel": float((st[0] / st[1]).sqrt()), "resid": float(res), "orth": float(orth), "ms": round(dt * 1e3, 3)}
        print(json.dumps(rec), flush=True)
    log.append(1)
    return orig(C, B_prev, max_sweeps=max_sweeps, tol=tol, return_stats=return_stats)


jacobi.warm_eigh = probe
center = (torch.rand(1000, generator=torch.Generator().manual_seed(1)) * 160 - 80).to(dev)
wf = StdWorkflow(CMAES(center_init=center, init_stdev=20.0, pop_size=10000), CEC2022TestSuit.create(1), graph=False)
st = wf.init(rnd.PRNGKey(2024, device=dev))
for _ in range(gens):
    st = wf.step(st)
torch.cuda.synchronize()
print("done", len(log))
