"""argsort of n f32 keys on one GPU: torch.sort (library radix), the LDS bitonic kernel,
the rocPRIM block radix kernel, the rank-by-counting kernel and the two-pass chunk-rank + co-rank
merge kernel (µs per call, graph-free,
200 reps; rows of 8 for the batched case)."""
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
                      "bitonic_us": t(lambda: ops.argsort_f32(k, 0)), "radix_us": t(lambda: ops.radix_argsort_f32(k, 0)),
                      "rank_us": t(lambda: ops.rank_argsort_f32(k, 0)), "rank_desc_us": t(lambda: ops.rank_argsort_f32(k, 1)),
                      "merge_us": t(lambda: ops.merge_argsort_f32(k, 0))}), flush=True)
for n in (20000, 30000, 32768, 50000, 65536):
    k = torch.randn(n, device="cuda")
    print(json.dumps({"n": n, "torch_sort_us": t(lambda: torch.sort(k, stable=True)),
                      "merge_us": t(lambda: ops.merge_argsort_f32(k, 0)), "merge_desc_us": t(lambda: ops.merge_argsort_f32(k, 1))}), flush=True)
for n in (1000, 10000):
    k = torch.randn(8, n, device="cuda")
    print(json.dumps({"batch": 8, "n": n, "torch_sort_us": t(lambda: torch.sort(k, dim=1, stable=True)),
                      "rank_us": t(lambda: ops.rank_argsort_f32(k, 0))}), flush=True)
