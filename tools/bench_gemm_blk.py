"""Microbenchmark of the blocked-planes bf16x6 GEMM (gemm_blk.hip) against gemm_ks and the
vendor f32 GEMM at the flagship's tall shapes; prints one JSON line per case (µs per call,
median of --reps event-timed calls after warm-up)."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from evoxmi import random as rnd  # noqa: E402
from evoxmi.ops import linalg  # noqa: E402


def timeit(fn, reps):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    ts.sort()
    return ts[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--shapes", default="10000x1000x1000,5000x1000x1000,10240x1024x1024")
    ap.add_argument("--only-blk", action="store_true")
    ap.add_argument("--only-h3", action="store_true", help="time the f16x3 product only (with EVOXMI_H3_CFG: one tile config)")
    args = ap.parse_args()
    dev = torch.device("cuda")
    # clocks up before the first timed case
    W = torch.randn(4096, 4096, device=dev)
    for _ in range(200):
        W @ W
    torch.cuda.synchronize()
    for sh in args.shapes.split(","):
        M, N, K = map(int, sh.split("x"))
        g = torch.Generator(device=dev).manual_seed(0)
        A = torch.randn(M, K, device=dev, generator=g)
        B = torch.randn(N, K, device=dev, generator=g)
        o = torch.randn(K, device=dev, generator=g)
        bias = torch.randn(N, device=dev, generator=g)
        sig = torch.tensor([0.5], device=dev)
        key = rnd.PRNGKey(3, device=dev)
        Ap = linalg.blk_planes(A)
        Bp = linalg.blk_planes(B)
        out = torch.empty(M, N, device=dev)
        res = {"shape": sh}
        Ah = linalg.h3_planes(A)
        Bh = linalg.h3_planes(B)
        res["h3_gemm_us"] = timeit(lambda: linalg.mm_h3(Ah, Bh, alpha_ptr=sig, bias_n=bias, out=out), args.reps)
        res["h3_pct_x3_ceiling"] = round(100 * 2.0 * M * N * K * 3 / (res["h3_gemm_us"] * 1e-6) / 2.5e15, 1)
        if args.only_h3:
            res["h3_cfg"] = os.environ.get("EVOXMI_H3_CFG", "auto")
            print(json.dumps({k: (round(v, 2) if isinstance(v, float) else v) for k, v in res.items()}), flush=True)
            continue
        res["blk_gemm_us"] = timeit(lambda: linalg.mm_blk(Ap, Bp, alpha_ptr=sig, bias_n=bias, out=out), args.reps)
        if args.only_blk:
            flops = 2.0 * M * N * K
            res["blk_pct_x6_ceiling"] = round(100 * flops * 6 / (res["blk_gemm_us"] * 1e-6) / 2.5e15, 1)
            print(json.dumps({k: (round(v, 2) if isinstance(v, float) else v) for k, v in res.items()}), flush=True)
            continue
        res["h3_split_A_us"] = timeit(lambda: linalg.h3_planes(A, sub_k=o, out=Ah), args.reps)
        res["h3_split_B_us"] = timeit(lambda: linalg.h3_planes(B, colscale=o, out=Bh), args.reps)
        if K % 4 == 0:
            res["h3_philox_A_us"] = timeit(lambda: linalg.normal_h3_planes(key, M, K, out=Ah), args.reps)
        res["blk_split_A_us"] = timeit(lambda: linalg.blk_planes(A, sub_k=o, out=Ap.t), args.reps)
        res["blk_split_B_us"] = timeit(lambda: linalg.blk_planes(B, colscale=o, out=Bp.t), args.reps)
        if K % 4 == 0:
            res["blk_philox_A_us"] = timeit(lambda: linalg.normal_blk_planes(key, M, K, out=Ap.t), args.reps)
        res["gemm_ks_us"] = timeit(lambda: linalg.mm(A, B, tb=True, alpha_ptr=sig, bias_n=bias, out=out), args.reps)
        res["torch_f32_us"] = timeit(lambda: torch.addmm(bias, A, B.t(), alpha=0.5, out=out), args.reps)
        flops = 2.0 * M * N * K
        res["blk_tflops_f32eq"] = round(flops / res["blk_gemm_us"] * 1e-6, 1)
        res["blk_pct_x6_ceiling"] = round(100 * flops * 6 / (res["blk_gemm_us"] * 1e-6) / 2.5e15, 1)
        print(json.dumps({k: (round(v, 2) if isinstance(v, float) else v) for k, v in res.items()}), flush=True)


if __name__ == "__main__":
    main()
