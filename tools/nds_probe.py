"""Per-front cost of the persistent NDS peel: random (n, m) objective sets, CPU front
count vs device time (hipEvent), optionally with EVOXMI_NDS_BLOCKS set by the caller."""
import json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from evoxmi.operators.selection import non_dominated_sort

for n, m in [(8192, 3), (8192, 2), (4096, 3), (16384, 3)]:
    f = torch.rand(n, m, generator=torch.Generator().manual_seed(n + m))
    fronts = int(non_dominated_sort(f).max()) + 1
    fc = f.cuda()
    for _ in range(3):
        non_dominated_sort(fc)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        non_dominated_sort(fc)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 10
    print(json.dumps({"n": n, "m": m, "fronts": fronts, "blocks_env": os.environ.get("EVOXMI_NDS_BLOCKS"), "ms": round(ms, 4), "us_per_front": round(ms * 1e3 / fronts, 2)}))
