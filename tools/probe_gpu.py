"""One-off hardware probe: library GEMM / eigh / sort rates that set the design budget."""
import time, torch, json
d = torch.device("cuda")
print(torch.__version__, torch.cuda.get_device_name(0), torch.version.hip)
p = torch.cuda.get_device_properties(0)
print("CUs", p.multi_processor_count, "mem", p.total_memory / 2**30, "arch", getattr(p, "gcnArchName", "?"))
def bench(fn, it=10):
    fn(); torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(it): fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / it * 1e3
res = {}
A = torch.randn(10000, 1000, device=d); B = torch.randn(1000, 1000, device=d)
ms = bench(lambda: A @ B); res["sgemm_10000x1000x1000_ms"] = ms; res["sgemm_TF"] = 2e10 / ms / 1e9
Y = torch.randn(5000, 1000, device=d)
ms = bench(lambda: Y.t() @ Y); res["syrk_1000x5000_ms"] = ms
C = torch.randn(1000, 1000, device=d); C = C @ C.t() / 1000 + torch.eye(1000, device=d)
for lib in ["default", "cusolver", "magma"]:
    try:
        if lib != "default": torch.backends.cuda.preferred_linalg_library(lib)
        ms = bench(lambda: torch.linalg.eigh(C), it=3); res[f"eigh1000_{lib}_ms"] = ms
    except Exception as e:
        res[f"eigh1000_{lib}_err"] = str(e)[:200]
f = torch.randn(10000, device=d)
res["sort10k_ms"] = bench(lambda: torch.sort(f), it=50)
res["randn_1e7_ms"] = bench(lambda: torch.randn(10000, 1000, device=d), it=20)
x = torch.randn(8192, 8192, device=d, dtype=torch.bfloat16)
ms = bench(lambda: x @ x, it=5); res["bf16_8192_TF"] = 2 * 8192**3 / ms / 1e9
print(json.dumps(res, indent=1))
