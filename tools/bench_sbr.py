"""Time the pieces of the sorted-block refinement eigensolver on a CMA-ES-like matrix
(d = 1000) and the full converged solve at several generation depths.

    python tools/bench_sbr.py [--n 1000] [--gens 4 15 40]
"""
import argparse
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from evoxmi.ops import sbr  # noqa: E402


def cma_like(n, gens, seed, dev):
    g = torch.Generator(device=dev).manual_seed(seed)
    mu = 5 * n
    w = math.log(mu + 0.5) - torch.log(torch.arange(1, mu + 1, dtype=torch.float64))
    w = (w / w.sum()).to(dev)
    mueff = float(w.sum() ** 2 / (w**2).sum())
    cmu = 2 * (mueff - 2 + 1 / mueff) / ((n + 2) ** 2 + mueff)
    C = torch.eye(n, dtype=torch.float64, device=dev)
    Bp = C.clone()
    for _ in range(gens):
        L = torch.linalg.cholesky(C)
        y = torch.randn(mu, n, generator=g, dtype=torch.float64, device=dev) @ L.T
        Bp = torch.linalg.eigh(C)[1]
        C = (1 - cmu) * C + cmu * (y.T * w) @ y
    return C.float(), Bp.float()


def timeit(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3  # µs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1000)
    ap.add_argument("--gens", type=int, nargs="*", default=[4, 15, 40])
    ap.add_argument("--block", type=int, default=16)
    a = ap.parse_args()
    dev = torch.device("cuda")
    C, B = cma_like(a.n, 20, 0, dev)
    A = sbr.sym_product(C, B)
    st = sbr.stats(A)
    res = {"stats_us": timeit(lambda: sbr.stats(A))}
    for bk in (16, 32, 64):
        perm, Q, dq = sbr.block_solve(A, 0, 2, bk)
        X = sbr.far(A, 0, perm, Q, dq, st, 0.3, bk)
        res.update({
            f"block{bk}_us": timeit(lambda: sbr.block_solve(A, 0, 2, bk)),
            f"far{bk}_us": timeit(lambda: sbr.far(A, 0, perm, Q, dq, st, 0.3, bk)),
            f"bq{bk}_us": timeit(lambda: sbr.bq(B, 0, perm, Q, bk)),
            f"refine_step{bk}_us": timeit(lambda: sbr.refine_step(C, A, B, st, 0, sbr.SBRConfig(block=bk)), reps=10),
        })
    res.update({"gemm_us": timeit(lambda: X @ X), "expm_us": timeit(lambda: sbr.expm_taylor6(X))})
    print(json.dumps(res), flush=True)
    for g in a.gens:
        C, B = cma_like(a.n, g, g, dev)
        sbr.eigh_warm(C, B, sbr.SBRConfig(block=a.block))
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        w, Bn, info = sbr.eigh_warm(C, B, sbr.SBRConfig(block=a.block))
        e.record()
        torch.cuda.synchronize()
        print(json.dumps({"gen": g, "ms": s.elapsed_time(e), "off_rel": info.off_rel, "jacobi": info.jacobi_sweeps,
                          "iters": info.refine_iters, "kappa0": info.kappa0, "fallback": info.fallback,
                          "history": info.history}), flush=True)


if __name__ == "__main__":
    main()
