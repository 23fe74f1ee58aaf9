import os, sys, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from evoxmi.ops import jacobi
dev = torch.device("cuda")
n = 1000
g = torch.Generator(device=dev).manual_seed(0)
Q, _ = torch.linalg.qr(torch.randn(n, n, device=dev, dtype=torch.float64, generator=g))
lam = torch.logspace(0, 3, n, device=dev, dtype=torch.float64)
Yr = torch.randn(2000, n, device=dev, dtype=torch.float64, generator=g) @ (Q * lam.sqrt()).T
C1 = (0.995 * (Q * lam) @ Q.T + 0.005 * (Yr.T @ Yr) / 2000).float()
Qf = Q.float().contiguous()
for _ in range(3):
    w, B, st = jacobi.warm_eigh(C1, Qf, max_sweeps=2, return_stats=True)
torch.cuda.synchronize()
print("rel_off", float((st[0] / st[1]).sqrt()))
