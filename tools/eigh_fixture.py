"""Run the flagship CMA-ES trajectory (bench.py's setup) eagerly and save the (C, B_prev) pair of
every device eigensolve that does not converge (capped, recovered or fallback) as a fixture for
tests/test_sbr_device_gpu.py — a debug tool, it reads the solve stats back after every generation.

    python tools/eigh_fixture.py --gens 40 [--simulate-rank 0 --world 8] --out gpurun_out/fix
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gens", type=int, default=40)
    ap.add_argument("--pop", type=int, default=10000)
    ap.add_argument("--dim", type=int, default=1000)
    ap.add_argument("--func", type=int, default=1)
    ap.add_argument("--seed", type=int, default=2024)
    ap.add_argument("--simulate-rank", type=int, default=None)
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--out", default="gpurun_out/eigh_fixture")
    ap.add_argument("--max-save", type=int, default=3)
    args = ap.parse_args()

    from evoxmi import config
    from evoxmi import random as rnd
    from evoxmi.algorithms import CMAES
    from evoxmi.ops import sbr_device
    from evoxmi.problems.numerical import CEC2022TestSuit
    from evoxmi.workflows import StdWorkflow

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    torch.manual_seed(0)
    key = rnd.PRNGKey(args.seed, device=dev)
    center = (torch.rand(args.dim, generator=torch.Generator().manual_seed(1)) * 160 - 80).to(dev)
    algo = CMAES(center_init=center, init_stdev=20.0, pop_size=args.pop)
    wf = StdWorkflow(algo, CEC2022TestSuit.create(args.func), graph=False)
    state = wf.init(key)
    if args.simulate_rank is not None:
        from evoxmi.parallel.context import SimulatedDistContext

        state = wf.enable_distributed(state, context=SimulatedDistContext(args.simulate_rank, args.world, algorithm=algo))

    last = {}
    orig = sbr_device.eigh_device

    def spy(C, B_prev, *a, **k):
        last["C"], last["B"] = C.detach().clone(), B_prev.detach().clone()
        last["iters"] = config.get("sbr_device_iters")
        out = orig(C, B_prev, *a, **k)
        last["stats"] = out[2]
        return out

    sbr_device.eigh_device = spy
    os.makedirs(args.out, exist_ok=True)
    saved = 0
    tol = float(config.get("eigh_tol"))
    for g in range(args.gens):
        last.clear()
        state = wf.step(state)
        if "stats" not in last:
            continue
        st = last["stats"].cpu().tolist()
        row = {"gen": g, "off_rel": st[0], "status": st[1], "iters": st[2], "fallback": st[3], "slots": last["iters"]}
        print(json.dumps(row), flush=True)
        if st[3] or st[0] > tol or st[1]:
            ws = [w for w in sbr_device._WS.values() if w.K == last["iters"]]
            if ws:
                w = ws[-1]
                h = w.hist.cpu().view(-1, 4)
                rel = (h[:, 0].clamp(min=0) / h[:, 1]).sqrt()
                kap = h[:, 0].clamp(min=0).sqrt() / (h[:, 3] - h[:, 2])
                print("   rel", [f"{v:.2e}" for v in rel.tolist()], flush=True)
                print("   kap", [f"{v:.2e}" for v in kap.tolist()], flush=True)
                print("   alpha", [f"{v:.3f}" for v in w.alpha.cpu().tolist()], flush=True)
                print("   ctrl", w.ctrl.cpu().view(-1, 8).tolist(), "st", w.st.cpu().tolist(), flush=True)
        if (st[3] or st[0] > tol or st[1]) and saved < args.max_save:
            path = os.path.join(args.out, f"gen{g:04d}.pt")
            torch.save({"C": last["C"].cpu(), "B_prev": last["B"].cpu(), "gen": g, "stats": st, "slots": last["iters"],
                        "variant": algo.graph_variant(g)}, path)
            print(f"saved {path}", flush=True)
            saved += 1


if __name__ == "__main__":
    main()
