"""Does D2HCopier.submit return before the GPU work it follows has finished (host time per
call, stream still busy afterwards)?"""
import sys, time, torch
sys.path.insert(0, "/root/repo")
from evoxmi.monitors.async_d2h import D2HCopier

a = torch.randn(4096, 4096, device="cuda")
x = torch.randn(10000, device="cuda")
c = D2HCopier()
for variant in ("arena", "fresh_pinned", "plain_copy_nonblocking"):
    ts, busy = [], 0
    for i in range(20):
        for _ in range(8):
            torch.mm(a, a)  # ~2 ms of GPU work queued
        t0 = time.perf_counter()
        if variant == "arena":
            c.submit(x)
        elif variant == "fresh_pinned":
            h = torch.empty(x.shape, dtype=x.dtype, pin_memory=True)
            h.copy_(x, non_blocking=True)
        else:
            h = torch.empty(x.shape, dtype=x.dtype)
            h.copy_(x, non_blocking=True)
        ts.append((time.perf_counter() - t0) * 1e6)
        busy += 0 if torch.cuda.current_stream().query() else 1
        torch.cuda.synchronize()
    print(f"{variant:24s} host us per submit: median {sorted(ts)[10]:8.1f} max {max(ts):8.1f}; GPU still busy after return: {busy}/20", flush=True)
