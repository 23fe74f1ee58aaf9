"""Device-controlled SBR schedule on the bench trajectory: per-generation refinement
iterations / off_rel for a given schedule length, and ms/generation.

    python tools/sbr_device_probe.py --iters 16 --gens 40
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=8)
    ap.add_argument("--gens", type=int, default=40)
    ap.add_argument("--mode", default="device")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--detail", action="store_true", help="per-iteration off_rel, κ, α and variant flags of every solve")
    a = ap.parse_args()
    os.environ["EVOXMI_SBR_DEVICE_ITERS"] = str(a.iters)
    os.environ["EVOXMI_SBR_MODE"] = a.mode
    from evoxmi import random as rnd
    from evoxmi.algorithms import CMAES
    from evoxmi.ops import sbr_device
    from evoxmi.problems.numerical import CEC2022TestSuit
    from evoxmi.workflows import StdWorkflow

    dev = torch.device("cuda")
    center = (torch.rand(1000, generator=torch.Generator().manual_seed(1)) * 160 - 80).to(dev)
    algo = CMAES(center_init=center, init_stdev=20.0, pop_size=10000)
    wf = StdWorkflow(algo, CEC2022TestSuit.create(1), graph=not a.no_graph)
    st = wf.init(rnd.PRNGKey(2024, device=dev))
    walls = []
    detail = []
    for g in range(a.gens):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        st = wf.step(st)
        torch.cuda.synchronize()
        walls.append((time.perf_counter() - t0) * 1e3)
        if a.detail:
            ws = list(sbr_device._WS.values())[-1]
            h = ws.hist.view(-1, 4).cpu().double()
            c = ws.ctrl.view(-1, 8).cpu()
            al = ws.alpha.cpu()
            its = []
            for j in range(ws.K + 1):
                off, dg, mn, mx = (float(x) for x in h[j])
                r = (max(off, 0) / dg) ** 0.5 if dg > 0 else float("nan")
                k = max(off, 0) ** 0.5 / (mx - mn) if mx > mn else float("inf")
                it = {"j": j - 1, "off_rel": float("%.3g" % r), "kappa": float("%.3g" % k)}
                if j >= 1:
                    cw = [int(x) for x in c[j - 1]]
                    if cw[0]:
                        break
                    it.update(far=1 - cw[1], damp=1 - cw[2], six=cw[4], ns=1 - cw[5], alpha=float("%.3g" % float(al[j])))
                its.append(it)
            detail.append({"gen": g + 1, "its": its})
    h = sbr_device.all_histories()
    rows = [{"gen": i + 1, "ms": round(walls[i], 3), "off_rel": float(h[i, 0]) if i < h.shape[0] else None,
             "iters": int(h[i, 2]) if i < h.shape[0] else None, "fallback": int(h[i, 3]) if i < h.shape[0] else None}
            for i in range(a.gens)]
    for r in rows:
        print(json.dumps(r))
    for d in detail:
        print(json.dumps(d))
    steady = walls[10:]
    print(json.dumps({"iters_schedule": a.iters, "mean_ms_gen_11_plus": round(sum(steady) / len(steady), 4),
                      "max_off_rel_gen_6_plus": max(r["off_rel"] for r in rows[5:] if r["off_rel"] is not None)}))


if __name__ == "__main__":
    main()
