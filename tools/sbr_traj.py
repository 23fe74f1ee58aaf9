"""Eigensolver variants on the covariance matrices of an actual bench run (CMA-ES pop
10 000, d 1000, CEC'22 F1): records (C, B_prev) of every generation, then decomposes each
with several SBR configurations and prints iterations / fallbacks / off-norm histories.

    python tools/sbr_traj.py [--gens 35] [--save 8 20 34]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from evoxmi import random as rnd  # noqa: E402
from evoxmi.algorithms import CMAES  # noqa: E402
from evoxmi.ops import sbr  # noqa: E402
from evoxmi.problems.numerical import CEC2022TestSuit  # noqa: E402
from evoxmi.workflows import StdWorkflow  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--gens", type=int, default=35)
ap.add_argument("--save", type=int, nargs="*", default=[])
ap.add_argument("--variants", default="16:0.3:1:3,16:0.5:1:3,16:0.3:1:0,64:0.3:0:3", help="block:thr_fac:local_theta:near_only,...")
a = ap.parse_args()
dev = torch.device("cuda")
rec = []
orig = sbr.eigh_warm


def hook(C, B_prev, cfg=None, plans=None):
    rec.append((C.detach().clone(), B_prev.detach().clone()))
    return orig(C, B_prev, sbr.SBRConfig(tol=cfg.tol if cfg else 1e-5, block=64))


sbr.eigh_warm = hook
torch.manual_seed(0)
prob = CEC2022TestSuit.create(1)
center = (torch.rand(1000, generator=torch.Generator().manual_seed(1)) * 160 - 80).to(dev)  # as bench.py
algo = CMAES(center_init=center, init_stdev=20.0, pop_size=10000)
wf = StdWorkflow(algo, prob, graph=False)
st = wf.init(rnd.PRNGKey(2024, device=dev))
for _ in range(a.gens):
    st = wf.step(st)
torch.cuda.synchronize()
sbr.eigh_warm = orig
print(f"recorded {len(rec)} decompositions", flush=True)
variants = [tuple(v.split(":")) for v in a.variants.split(",")]
tot = {v: [0, 0] for v in variants}
for g, (C, B) in enumerate(rec):
    out = {"gen": g}
    for v in variants:
        bk, thr, theta, near = v
        sbr.LOCAL_THETA = float(theta)
        w, Bn, info = orig(C, B, sbr.SBRConfig(block=int(bk), thr_fac=float(thr), near_only=float(near)))
        tot[v][0] += info.refine_iters + info.jacobi_sweeps
        tot[v][1] += int(info.fallback)
        out[":".join(v)] = [info.refine_iters, info.jacobi_sweeps, int(info.fallback), info.damped,
                              [f"{h[0][0]}{h[1]:.1e}" for h in info.history]]
    print(json.dumps(out), flush=True)
print(json.dumps({":".join(k): v for k, v in tot.items()}), flush=True)
if a.save:
    os.makedirs("gpurun_out/sbr16", exist_ok=True)
    torch.save({g: (rec[g][0].cpu(), rec[g][1].cpu()) for g in a.save if g < len(rec)}, "gpurun_out/sbr16/mats.pt")
