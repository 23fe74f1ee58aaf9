"""How small are the eigensolver's far generators in settled CMA-ES solves, and how tight is the
free bound the device schedule can test on the device (X² GEMM's diagonal stats)?  Runs the flagship
(pop 10 000, CEC'22 F1, d 1000) eagerly; for the solves of generations ≥ --from it replays the solve
slot by slot on a probe workspace and prints per refinement iteration: off_rel after it, the
upper bound U ≥ ‖X‖₂² from the stats, the true ‖X‖₂ and ‖X‖_F.

    python tools/xnorm_probe.py [--gens 32] [--from 28]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gens", type=int, default=32)
    ap.add_argument("--from", dest="first", type=int, default=28)
    a = ap.parse_args()
    from evoxmi import random as rnd
    from evoxmi.algorithms import CMAES
    from evoxmi.ops import _ext, sbr_device
    from evoxmi.problems.numerical import CEC2022TestSuit
    from evoxmi.workflows import StdWorkflow

    dev = torch.device("cuda")
    gen = [0]
    orig = sbr_device.eigh_device

    def probe(C, B_prev, cfg=None, iters=None):
        if gen[0] >= a.first:
            # xgate on: the X² GEMM writes the diagonal stats the bound is read from
            ws = sbr_device.DeviceSBR(C.shape[0], C.device, sbr_device.device_config(), 7, sbr_device.FULL_SLOTS, True, None)
            ops = _ext.ops()
            ops.sbr_dev_copy(B_prev.contiguous(), ws.B, ws.never)
            ws._btcb(C, ws.never)
            ws._ctrl(-1, C)
            for j in range(ws.K):
                ws._iteration(j, C)
                torch.cuda.synchronize()
                c = ws.ctrl[sbr_device.CW * j : sbr_device.CW * j + 8].cpu().tolist()
                if c[0]:
                    break
                h = ws.hist.view(-1, 4)[j + 1].cpu()
                p = ws.part2.view(-1, 4).double().cpu() if ws.part2 is not None else None
                X = ws.X.double()
                print(json.dumps({"gen": gen[0], "iter": j, "far": int(c[1] == 0), "order6": c[4], "ns": int(c[5] == 0),
                                  "alpha": float(ws.alpha[j + 1]), "off_rel_after": float((h[0] / h[1]).sqrt()),
                                  "U_bound": float((C.shape[0] * p[:, 1].sum()).sqrt()) if (c[1] == 0 and p is not None) else None,
                                  "X_2norm": float(torch.linalg.matrix_norm(X, 2)) if c[1] == 0 else None,
                                  "X_fro": float(torch.linalg.matrix_norm(X)) if c[1] == 0 else None}), flush=True)
        return orig(C, B_prev, cfg, iters)

    sbr_device.eigh_device = probe
    center = (torch.rand(1000, generator=torch.Generator().manual_seed(1)) * 160 - 80).to(dev)
    algo = CMAES(center_init=center, init_stdev=20.0, pop_size=10000)
    wf = StdWorkflow(algo, CEC2022TestSuit.create(1), graph=False)
    st = wf.init(rnd.PRNGKey(2024, device=dev))
    for g in range(a.gens):
        gen[0] = g
        st = wf.step(st)


if __name__ == "__main__":
    main()
