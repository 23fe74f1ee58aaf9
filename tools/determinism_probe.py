"""Bitwise determinism of the pieces of the SBR solve and of plain f32 GEMMs."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from evoxmi.ops import sbr  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from bench_sbr import cma_like  # noqa: E402

for n in (64, 1000):
    torch.manual_seed(0)
    X = torch.randn(n, n, device="cuda")
    Y = [X @ X for _ in range(20)]
    print(n, "gemm deterministic:", all(torch.equal(Y[0], y) for y in Y), flush=True)
    C, B = cma_like(n, 6, 3, torch.device("cuda"))
    outs = []
    for r in range(4):
        w, Bn, info = sbr.eigh_warm(C, B, sbr.SBRConfig(), plans={})
        outs.append((w.clone(), Bn.clone(), info.refine_iters, info.off_rel))
    print(n, "eigh deterministic:", all(torch.equal(outs[0][1], o[1]) for o in outs), [(o[2], o[3]) for o in outs], flush=True)
    A = sbr.sym_product(C, B)
    st = sbr.stats(A)
    r = [sbr.block_solve(A, 0, 2, 16) for _ in range(5)]
    print(n, "block deterministic:", all(torch.equal(r[0][1], x[1]) and torch.equal(r[0][0], x[0]) for x in r), flush=True)
    p, Q, dq = r[0]
    xs = [sbr.far(A, 0, p, Q, dq, st, 0.3, 16) for _ in range(5)]
    print(n, "far deterministic:", all(torch.equal(xs[0], x) for x in xs), flush=True)
