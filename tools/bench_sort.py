"""argsort of n f32 keys on one GPU: torch.sort (library radix), the LDS bitonic kernel
and the rocPRIM block radix kernel (µs per call, graph-free, 200 reps)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from evoxmi.ops import _ext  # noqa: E402


def t(fn, reps=200):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return round(s.elapsed_time(e) / reps * 1e3, 2)


ops = _ext.ops()
for n in (1000, 2048, 4096, 8192, 10000, 16384):
    k = torch.randn(n, device="cuda")
    print(json.dumps({"n": n, "torch_sort_us": t(lambda: torch.sort(k, stable=True)),
                      "bitonic_us": t(lambda: ops.argsort_f32(k, 0)), "radix_us": t(lambda: ops.radix_argsort_f32(k, 0))}), flush=True)
