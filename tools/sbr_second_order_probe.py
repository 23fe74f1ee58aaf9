"""Round-6 convergence probe of the sorted-block refinement (profiles/r6_sbr_convergence_analysis.txt).

Reads C and the warm-start basis of flagship solves dumped by scratch7/it.py on the GPU box
(gpurun_out/dl/mat_<solve>.pt, torch.save of CPU tensors written by this repo) and replays the
reference steps of evoxmi/ops/sbr.py in float64 on the CPU."""
import math, sys, torch
ROOT = __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__)))
sys.path.insert(0, ROOT)
from evoxmi.ops import sbr
torch.set_num_threads(8)
def r_of(st):
    off, dg, mn, mx = [float(x) for x in st[:4]]
    return math.sqrt(max(off, 0) / dg)
def step(C, A, B, st, it, second, thr=0.3, theta=0.0, sweeps=2, sb=32, ns=True, corr_scale=1.0):
    shift = (it % 2) * (sb // 2)
    perm, Q, dq = sbr.block_solve16_ref(A, shift, sweeps, sb)
    p = perm.long()
    Qf = sbr._blockdiag16(Q, A.shape[0])
    X = sbr.far16_ref(A, perm, Q, dq, st, thr, theta)
    if second:
        A1 = Qf.T @ A[p][:, p] @ Qf
        E = A1 - torch.diag(torch.diagonal(A1))
        M = E @ X
        Cm = M + M.T
        den = dq[None, :] - dq[:, None]
        mask = X != 0
        X = X + torch.where(mask, corr_scale * 0.5 * Cm / torch.where(mask, den, torch.ones_like(den)), torch.zeros_like(X))
        X = 0.5 * (X - X.T)
    V = torch.linalg.matrix_exp(X)
    Bn = B[:, p] @ Qf @ V
    if ns:
        Bn = sbr.newton_schulz(Bn)
    A, st = sbr.sym_product_stats(C, Bn)
    return A, Bn, st
for mat in ("mat_40", "mat_10"):
    d = torch.load(f"{ROOT}/gpurun_out/dl/{mat}.pt", weights_only=True)
    for second in (False, True):
        C, B = d["C"].double(), d["B_prev"].double()
        A, st = sbr.sym_product_stats(C, B)
        rs = [r_of(st)]
        for it in range(5):
            A, B, st = step(C, A, B, st, it, second, theta=(1.0 if it >= 2 else 0.0))
            rs.append(r_of(st))
        print(mat, "second" if second else "first ", " ".join(f"{x:.1e}" for x in rs), "| ratios", " ".join(f"{rs[i+1]/rs[i]:.2f}" for i in range(5)), flush=True)
print("grid")
d = torch.load(ROOT + "/gpurun_out/dl/mat_40.pt", weights_only=True)
import itertools
for thr, tf, second, sweeps in itertools.product((0.3, 0.1, 0.05), (0, 2), (False, True), (2, 3)):
    C, B = d["C"].double(), d["B_prev"].double()
    A, st = sbr.sym_product_stats(C, B)
    rs = [r_of(st)]
    for it in range(4):
        A, B, st = step(C, A, B, st, it, second, thr=thr, theta=(1.0 if it >= tf else 0.0), sweeps=sweeps, ns=it < 2)
        rs.append(r_of(st))
    print(f"thr {thr} theta_from {tf} second {int(second)} sweeps {sweeps}:", " ".join(f"{x:.1e}" for x in rs), flush=True)
