"""Microbenchmark of the flagship's f32 GEMM shapes: gemm_ks (hand-written MFMA) in both
precision modes ('x6': exact three-way bf16 split, six bf16 MFMA products; 'f32': f32 MFMA)
vs torch.mm (hipBLASLt).  Device time per call from HIP events over back-to-back calls;
``err_x6`` / ``err_f32`` = max |C − C_fp64| / Σ_k |a·b| of one call (the test bound is 2e-6).

    python tools/bench_gemm.py [--reps 100] [--tile 0]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from evoxmi.ops import _ext, linalg  # noqa: E402


def timeit(fn, reps, warm=10):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps  # µs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=100)
    ap.add_argument("--tile", type=int, default=0, help="force the gemm_ks tile (2/3/4 ×16), 0 = heuristic")
    a = ap.parse_args()
    _ext.ops().gemm_ks_set_tile(a.tile)
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    n = 1000
    A = torch.randn(n, n, device=dev, generator=g)
    B = torch.randn(n, n, device=dev, generator=g)
    X = torch.randn(n, n, device=dev, generator=g)
    X = (X - X.t()) / 2
    Y = torch.randn(5000, n, device=dev, generator=g)
    Z = torch.randn(10000, n, device=dev, generator=g)
    bias = torch.randn(n, device=dev, generator=g)
    out = torch.empty(n, n, device=dev)
    out_t = torch.empty(10000, n, device=dev)
    cases = [
        ("1000^3 A·Bt (NT)", 2 * n**3, lambda: linalg.mm(A, B, tb=True, out=out), lambda: torch.mm(A, B.t(), out=out)),
        ("1000^3 A·B (NN)", 2 * n**3, lambda: linalg.mm(A, B, out=out), lambda: torch.mm(A, B, out=out)),
        ("1000^3 At·B (TN)", 2 * n**3, lambda: linalg.mm(A, B, ta=True, out=out), lambda: torch.mm(A.t(), B, out=out)),
        ("1000^3 X·X sym (NT, -X·Xt)", 2 * n**3, lambda: linalg.mm(X, X, tb=True, mode=1, alpha=-1.0, out=out),
         lambda: torch.mm(X, X, out=out)),
        ("1000^3 At·B sym (TN)", 2 * n**3, lambda: linalg.mm(A, A, ta=True, mode=1, out=out), lambda: torch.mm(A.t(), A, out=out)),
        ("1000^3 skew X2·X (NT)", 2 * n**3, lambda: linalg.mm(A, X, tb=True, mode=2, alpha=-1.0, out=out),
         lambda: torch.mm(A, X, out=out)),
        ("1000x1000x5000 Yt·Y sym (TN)", 2 * n * n * 5000, lambda: linalg.mm(Y, Y, ta=True, mode=1, out=out),
         lambda: torch.mm(Y.t(), Y, out=out)),
        ("10000x1000x1000 Z·Bt + bias (NT)", 2 * 10000 * n * n, lambda: linalg.mm(Z, B, tb=True, bias_n=bias, out=out_t),
         lambda: torch.addmm(bias, Z, B.t(), out=out_t)),
    ]
    from evoxmi import config

    # accuracy of both modes on the NT product (fp64 reference on the device)
    Ad, Bd = A.double(), B.double()
    R = Ad @ Bd.t()
    Bound = Ad.abs() @ Bd.abs().t()
    errs = {}
    for prec in ("x6", "f32"):
        with config.override(gemm_prec=prec):
            C = linalg.mm(A, B, tb=True)
        errs[prec] = float(((C.double() - R).abs() / Bound).max())
    print(json.dumps({"err_x6": errs["x6"], "err_f32": errs["f32"]}), flush=True)
    rows = []
    for name, flops, f_ks, f_t in cases:
        t = {}
        for prec in ("x6", "f32"):
            with config.override(gemm_prec=prec):
                t[prec] = timeit(f_ks, a.reps)
        t_t = timeit(f_t, a.reps)
        rows.append({"case": name, "x6_us": round(t["x6"], 2), "f32_us": round(t["f32"], 2), "torch_us": round(t_t, 2),
                     "x6_tflops": round(flops / t["x6"] / 1e6, 1), "f32_tflops": round(flops / t["f32"] / 1e6, 1),
                     "torch_tflops": round(flops / t_t / 1e6, 1), "x6_vs_torch": round(t_t / t["x6"], 3)})
        print(json.dumps(rows[-1]), flush=True)


if __name__ == "__main__":
    main()
