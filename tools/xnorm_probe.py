"""How small are the eigensolver's far generators in settled CMA-ES solves, and how tight is the
free bound the device schedule can test on the device (X² GEMM's diagonal stats)?  Runs the flagship
(pop 10 000, CEC'22 F1, d 1000) for --gens generations, then replays a few solves slot by slot and
prints per refinement iteration: the upper bound U ≥ ‖X‖₂² from the stats, the true ‖X‖₂ and ‖X‖_F.

    python tools/xnorm_probe.py [--gens 30] [--solves 3]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gens", type=int, default=30)
    ap.add_argument("--solves", type=int, default=3)
    a = ap.parse_args()
    from evoxmi import random as rnd
    from evoxmi.algorithms import CMAES
    from evoxmi.ops import sbr_device
    from evoxmi.problems.numerical import CEC2022TestSuit
    from evoxmi.workflows import StdWorkflow

    dev = torch.device("cuda")
    center = (torch.rand(1000, generator=torch.Generator().manual_seed(1)) * 160 - 80).to(dev)
    algo = CMAES(center_init=center, init_stdev=20.0, pop_size=10000)
    wf = StdWorkflow(algo, CEC2022TestSuit.create(1), graph=True)
    st = wf.init(rnd.PRNGKey(2024, device=dev))
    for g in range(a.gens + a.solves):
        if g >= a.gens:
            alg = st.get_child_state("algorithm")
            C = torch.triu(alg.C) + torch.triu(alg.C, 1).T
            ws = sbr_device.workspace(1000, dev, sbr_device.device_config(), 7, sbr_device.FULL_SLOTS, False, None)
            ws.solve(C.contiguous(), alg.B.contiguous())  # warm the workspace
            from evoxmi.ops import _ext

            ops = _ext.ops()
            ops.sbr_dev_copy(alg.B.contiguous(), ws.B, ws.never)
            ws._btcb(C.contiguous(), ws.never)
            ws._ctrl(-1, C)
            for j in range(ws.K):
                ws._iteration(j, C)
                torch.cuda.synchronize()
                c = ws.ctrl[sbr_device.CW * j : sbr_device.CW * j + 9].cpu().tolist()
                if c[0] or c[1]:
                    continue
                p = ws.part2.view(-1, 4).double().cpu()
                U = float((1000 * p[:, 1].sum()).sqrt())
                X = ws.X.double()
                print(json.dumps({"gen": g, "iter": j, "U_bound_X2norm2": U, "X_2norm": float(torch.linalg.matrix_norm(X, 2)),
                                  "X_fro": float(torch.linalg.matrix_norm(X)), "alpha": float(ws.alpha[j + 1]),
                                  "order6": c[4], "skip_vt": c[8], "off_rel": float(ws.hist.view(-1, 4)[j + 1, 0].sqrt() / ws.hist.view(-1, 4)[j + 1, 1].sqrt())}),
                      flush=True)
        st = wf.step(st)


if __name__ == "__main__":
    main()
