"""Round-6 probe: the damping cap tau of the far step on flagship matrices dumped by scratch7/it.py
(CPU replay of evoxmi/ops/sbr.py; profiles/r6_sbr_convergence_analysis.txt)."""
import math, sys, torch
ROOT = __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__)))
sys.path.insert(0, ROOT)
from evoxmi.ops import sbr
torch.set_num_threads(8)
def r_of(st):
    off, dg, mn, mx = [float(x) for x in st[:4]]
    return math.sqrt(max(off, 0) / dg), math.sqrt(max(off, 0)) / (mx - mn)
for mat in ("mat_10", "mat_40"):
    d = torch.load(f"{ROOT}/gpurun_out/dl/{mat}.pt", weights_only=True)
    for tau in (0.5, 0.75, 1.0, 1.5, 2.0, 3.0):
        cfg = sbr.SBRConfig(thr_fac=0.3, block_sweeps=2, block=32, damp_tau=tau)
        C, B = d["C"].float(), d["B_prev"].float()
        A, st = sbr.sym_product_stats(C, B)
        rs = [r_of(st)[0]]; al = []
        for it in range(5):
            r, k = r_of(st)
            damp = it == 0 or k > cfg.damp_kappa
            A, B, st, a = sbr._refine_core(C, A, B, st, (it % 2) * 16, True, damp, cfg, theta=(1.0 if k <= 0.05 else 0.0), order=6)
            rs.append(r_of(st)[0]); al.append(float(a.reshape(-1)[0]))
        print(mat, f"tau {tau}", " ".join(f"{x:.1e}" for x in rs), "| alpha", " ".join(f"{x:.2f}" for x in al), flush=True)
