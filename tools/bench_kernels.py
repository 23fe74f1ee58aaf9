"""Micro-benchmarks of the flagship kernels vs the ROCm libraries (run on the GPU box)."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from evoxmi.ops import jacobi  # noqa: E402
from evoxmi.ops.linalg import Operand, gemm  # noqa: E402
from evoxmi.ops.sort import argsort  # noqa: E402


def t(fn, it=20):
    fn()
    torch.cuda.synchronize()
    s = time.perf_counter()
    for _ in range(it):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - s) / it * 1e3


dev = torch.device("cuda")
res = {}
A = torch.randn(10000, 1000, device=dev)
B = torch.randn(1000, 1000, device=dev)
from evoxmi.ops import _ext
ops = _ext.ops()
D = torch.rand(1000, device=dev)
for cfg in (-1, 0, 3, 4, 5, 6, 7):
    ops.gemm_set_config(cfg)
    res[f"gemm_nt_10000x1000x1000_cfg{cfg}_ms"] = t(lambda: gemm(Operand(A), Operand(B), 10000, 1000, 1000))
    res[f"gemm_nt_pro_10000x1000x1000_cfg{cfg}_ms"] = t(lambda: gemm(Operand(A, kscale=D), Operand(B), 10000, 1000, 1000))
    idx0 = torch.randperm(10000, device=dev)[:5000].to(torch.int32)
    res[f"gemm_tn_gather_split8_cfg{cfg}_ms"] = t(lambda: gemm(Operand(A, rc=True, gather=idx0, sub=D), Operand(A, rc=True, gather=idx0, sub=D), 1000, 1000, 5000, splits=8))
    res[f"gemm_1024_nn_cfg{cfg}_ms"] = t(lambda: gemm(Operand(B), Operand(B, rc=True), 1000, 1000, 1000))
ops.gemm_set_config(-1)
res["torch_mm_10000x1000x1000_ms"] = t(lambda: A @ B.T)
idx = torch.randperm(10000, device=dev)[:5000].to(torch.int32)
m = torch.randn(1000, device=dev)
w = torch.rand(5000, device=dev)
for sp in (4, 8, 16):
    res[f"gemm_tn_gather_1000x1000x5000_split{sp}_ms"] = t(lambda: gemm(Operand(A, rc=True, gather=idx, sub=m, kw=w), Operand(A, rc=True, gather=idx, sub=m), 1000, 1000, 5000, splits=sp))
Y = A[:5000]
res["torch_syrk_ms"] = t(lambda: Y.T @ Y)
f = torch.randn(10000, device=dev)
res["argsort_lds_10000_ms"] = t(lambda: argsort(f))
res["torch_sort_10000_ms"] = t(lambda: torch.sort(f))
n = 1000
Q, _ = torch.linalg.qr(torch.randn(n, n, device=dev, dtype=torch.float64))
lam = torch.logspace(0, 3, n, device=dev, dtype=torch.float64)
C0 = (Q * lam) @ Q.T
Yr = torch.randn(2000, n, device=dev, dtype=torch.float64) @ (Q * lam.sqrt()).T
C1 = (0.995 * C0 + 0.005 * (Yr.T @ Yr) / 2000).float()
Qf = Q.float().contiguous()
for sw in (1, 2, 3):
    res[f"warm_eigh_{sw}sweep_ms"] = t(lambda: jacobi.warm_eigh(C1, Qf, max_sweeps=sw), it=5)
    _, _, st = jacobi.warm_eigh(C1, Qf, max_sweeps=sw, return_stats=True)
    res[f"warm_eigh_{sw}sweep_rel_off"] = float((st[0] / st[1]).sqrt())
res["cold_eigh_jacobi_ms"] = t(lambda: jacobi.eigh(C1), it=3)
res["torch_eigh_ms"] = t(lambda: torch.linalg.eigh(C1), it=3)
print(json.dumps(res, indent=1))
