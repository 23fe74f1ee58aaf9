"""Round-6 convergence probe of the sorted-block refinement (profiles/r6_sbr_convergence_analysis.txt).

Reads C and the warm-start basis of flagship solves dumped by scratch7/it.py on the GPU box
(gpurun_out/dl/mat_<solve>.pt, torch.save of CPU tensors written by this repo) and replays the
reference steps of evoxmi/ops/sbr.py in float64 on the CPU."""
import math, sys, torch
ROOT = __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__)))
sys.path.insert(0, ROOT)
from evoxmi.ops import sbr
torch.set_num_threads(8)
d = torch.load(ROOT + "/gpurun_out/dl/mat_40.pt", weights_only=True)
C, B = d["C"].double(), d["B_prev"].double()
cfg = sbr.SBRConfig(thr_fac=0.3, block_sweeps=2, block=32)
A, st = sbr.sym_product_stats(C, B)
def classes(A, label):
    dg = torch.diagonal(A)
    n = A.shape[0]
    spread = float(dg.max() - dg.min())
    g = (dg[None, :] - dg[:, None]).abs() / (spread / n)
    off = A - torch.diag(dg)
    tot = float((off ** 2).sum())
    # rank distance
    rk = torch.empty(n, dtype=torch.long); rk[torch.argsort(dg)] = torch.arange(n)
    rd = (rk[None, :] - rk[:, None]).abs()
    out = []
    for lo, hi in [(0, 1), (1, 4), (4, 16), (16, 64), (64, 1e9)]:
        m = (g >= lo) & (g < hi) & (rd > 0)
        out.append(f"gap[{lo},{hi}) {float((off[m] ** 2).sum()) / tot:.2f}")
    outr = []
    for lo, hi in [(1, 2), (2, 8), (8, 32), (32, 128), (128, 10000)]:
        m = (rd >= lo) & (rd < hi)
        outr.append(f"rank[{lo},{hi}) {float((off[m] ** 2).sum()) / tot:.2f}")
    print(label, f"off_rel {math.sqrt(tot / float((dg**2).sum())):.1e}", " ".join(out), "|", " ".join(outr))
    print("   spread", spread, "diag range", float(dg.min()), float(dg.max()), "median gap/avg", float(torch.diff(torch.sort(dg).values).median()) / (spread / n))
classes(A, "warm start")
for it in range(3):
    A, B, st, _ = sbr._refine_core(C, A, B, st, (it % 2) * 16, it < 2, False, cfg, theta=(1.0 if it >= 2 else 0.0), order=6)
    classes(A, f"after it {it}")
