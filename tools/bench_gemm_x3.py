"""bf16x3 vs bf16x6 on the eigensolver's 1000³ product shapes (gemm_ks.hip PREC 3 vs 1): device
µs per call (HIP events, back-to-back calls) and the max error relative to Σ_k|a·b| (fp64
reference).  The x3 products are used only for corrections (exp(αX) − I terms, T·(BᵀB − I)).

    python tools/bench_gemm_x3.py [--reps 200] [--n 1000]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from evoxmi.ops import linalg  # noqa: E402


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
    return e0.elapsed_time(e1) * 1e3 / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=200)
    ap.add_argument("--n", type=int, default=1000)
    a = ap.parse_args()
    n, dev = a.n, "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    A = torch.randn(n, n, device=dev, generator=g)
    B = torch.randn(n, n, device=dev, generator=g)
    X = torch.randn(n, n, device=dev, generator=g)
    X = (X - X.t()) / 2
    out = torch.empty(n, n, device=dev)
    cases = {
        "NT": dict(A=A, B=B, tb=True),
        "NN": dict(A=A, B=B),
        "TN": dict(A=A, B=B, ta=True),
        "XXt sym": dict(A=X, B=X, tb=True, mode=1, alpha=-1.0),
        "skew X2X": dict(A=-(X @ X.t()), B=X, tb=True, mode=2, alpha=-1.0),
        "NT +Cin": dict(A=A, B=B, tb=True, beta=1.0, Cin=B),
    }
    rows = []
    for name, kw in cases.items():
        kw = dict(kw)
        Am, Bm = kw.pop("A"), kw.pop("B")
        ref_a = (Am.t() if kw.get("ta") else Am).double()
        ref_b = (Bm.t() if kw.get("tb") else Bm).double()
        R = kw.get("alpha", 1.0) * (ref_a @ ref_b)
        if "Cin" in kw:
            R = R + kw["beta"] * kw["Cin"].double()
        S = ref_a.abs() @ ref_b.abs()
        row = {"case": name}
        for prec in (None, "x3"):
            f = lambda: linalg.mm(Am, Bm, out=out, prec=prec, **kw)  # noqa: E731
            us = timeit(f, a.reps)
            f()
            torch.cuda.synchronize()
            err = float(((out.double() - R).abs() / S).max())
            row["us_" + (prec or "x6")] = round(us, 2)
            row["err_" + (prec or "x6")] = err
        rows.append(row)
        print(json.dumps(row), flush=True)
    # a rank's column block of the same products under a column-distributed eigensolver (W = 2 / 4 / 8):
    # the 1000² output already holds one 64 × 64 tile per CU, so a narrower output keeps each tile's
    # serial K loop and only idles CUs — the evidence for keeping the d = 1000 solve replicated
    for w in (2, 4, 8):
        nc = n // w
        Bn = B[:, :nc].contiguous()
        on = torch.empty(n, nc, device=dev)
        for prec in (None, "x3"):
            us = timeit(lambda: linalg.mm(A, Bn, out=on, prec=prec), a.reps)
            print(json.dumps({"case": f"NN column block 1000x{nc}x1000 (W={w})", "prec": prec or "x6", "us": round(us, 2)}), flush=True)
    # diag_add: BᵀB − I on an orthogonal B
    Q, _ = torch.linalg.qr(torch.randn(n, n, device=dev, generator=g, dtype=torch.float64))
    Qf = Q.float()
    linalg.mm(Qf, Qf, ta=True, mode=1, out=out, diag_add=-1.0)
    E = Qf.double().t() @ Qf.double() - torch.eye(n, device=dev, dtype=torch.float64)
    print(json.dumps({"case": "BtB-I diag_add", "max_abs_err": float((out.double() - E).abs().max()),
                      "max_abs_E": float(E.abs().max())}), flush=True)


if __name__ == "__main__":
    main()
