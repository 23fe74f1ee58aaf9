"""CEC'22 F1 / F4 evaluation at pop 10 000, d 1000: fused rotation GEMM + row-terms epilogue
vs rotation GEMM (Z written) + basic-function kernel."""
import sys, torch
sys.path.insert(0, "/root/repo")
from evoxmi.ops import linalg
from evoxmi.ops import numerical as nops
from evoxmi.problems.numerical import CEC2022TestSuit
from evoxmi.problems.numerical.cec2022 import _rowterms

X = torch.rand(10000, 1000, device="cuda") * 160 - 80


def timeit(f, n=50):
    f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        f()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


for fn, fid in ((1, 0), (4, 3)):
    p = CEC2022TestSuit.create(fn)
    c = p._consts(1000, X.device)
    o, M = c["Os"][:1000].contiguous(), c["M"]
    fused = lambda: _rowterms(X, o, M, 1.0, fid)
    gemm_only = lambda: linalg.plain_nt(X, M, alpha=1.0, a_sub_k=o)
    Z = gemm_only()
    basic_only = lambda: nops.cec_basic(Z, fid, None, 0, 1000, None, 1.0, None, 0)
    print(f"F{fn}: fused {timeit(fused):7.1f} us   GEMM (Z written) {timeit(gemm_only):7.1f} us + basic kernel {timeit(basic_only):6.1f} us", flush=True)
