import sys, math, torch
sys.path.insert(0, '/root/repo')
from evoxmi.ops import sbr
n = 500
g = torch.Generator(device="cuda").manual_seed(3)
C = torch.eye(n, device="cuda"); B = torch.eye(n, device="cuda")
eye = torch.eye(n, device="cuda", dtype=torch.float64)
worst = 0
for k in range(40):
    Y = torch.randn(1000, n, device="cuda", generator=g)
    C = 0.99 * C + 0.01 * (Y.T @ Y) / 1000
    w, B, info = sbr.eigh_warm(C, B)
    Bd = B.double()
    res = ((Bd * w.double()) @ Bd.T - C.double()).norm() / C.double().norm()
    orth = (Bd.T @ Bd - eye).norm() / math.sqrt(n)
    A = Bd.T @ C.double() @ Bd
    off = (A - torch.diag(torch.diagonal(A))).norm() / torch.diagonal(A).norm()
    worst = max(worst, res.item())
    if k % 5 == 4 or res.item() > 1.8e-5:
        print(k, f"res {res.item():.3e} orth {orth.item():.3e} off64 {off.item():.3e} info.off {info.off_rel:.3e} iters {info.refine_iters}", flush=True)
print("worst", worst)
