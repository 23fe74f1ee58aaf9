"""Round-6 probe: a near-only (block step only) final refinement iteration vs a far one, on the
flagship matrices dumped by scratch7/it.py (CPU replay of evoxmi/ops/sbr.py; profiles/NOTES.md)."""
import math, sys, torch
ROOT = __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__)))
sys.path.insert(0, ROOT)
from evoxmi.ops import sbr
torch.set_num_threads(8)
def r_of(st):
    off, dg, mn, mx = [float(x) for x in st[:4]]
    return math.sqrt(max(off, 0) / dg)
for mat in ("mat_40", "mat_41"):
    d = torch.load(f"{ROOT}/gpurun_out/dl/{mat}.pt", weights_only=True)
    cfg = sbr.SBRConfig(thr_fac=0.3, block_sweeps=2, block=32)
    for dtype in (torch.float64, torch.float32):
        C, B = d["C"].to(dtype), d["B_prev"].to(dtype)
        A, st = sbr.sym_product_stats(C, B)
        rs = [r_of(st)]
        for it in range(3):
            A, B, st, _ = sbr._refine_core(C, A, B, st, (it % 2) * 16, it < 2, False, cfg, theta=(1.0 if it >= 2 else 0.0), order=6)
            rs.append(r_of(st))
        A3, B3, st3 = A, B, st
        # 4th: far (as now) vs near-only with either shift, and two near-only
        Af, Bf, stf, _ = sbr._refine_core(C, A3, B3, st3, 16, False, False, cfg, theta=1.0, order=4)
        An, Bn, stn, _ = sbr._refine_core(C, A3, B3, st3, 16, False, False, cfg, far_on=False)
        An0, Bn0, stn0, _ = sbr._refine_core(C, A3, B3, st3, 0, False, False, cfg, far_on=False)
        An2, Bn2, stn2, _ = sbr._refine_core(C, An, Bn, stn, 0, False, False, cfg, far_on=False)
        print(mat, dtype, " ".join(f"{x:.1e}" for x in rs), f"| 4th far {r_of(stf):.1e} near(s16) {r_of(stn):.1e} near(s0) {r_of(stn0):.1e} near,near {r_of(stn2):.1e}", flush=True)
