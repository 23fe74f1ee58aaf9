"""Per-generation kernel timeline from a rocprofv3 kernel_trace.csv: generations are cut at
a marker kernel (default philox_fill); prints the last full generation with gaps, and a
summary (wall, busy, idle) of every generation.

    python tools/ktrace_gen.py TRACE.csv [--marker philox_fill] [--show -2]
"""
import argparse
import csv

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("--marker", default="philox_fill")
ap.add_argument("--show", type=int, default=-2)
ap.add_argument("--quiet", action="store_true")
a = ap.parse_args()
rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if a.marker in r["Kernel_Name"]]
gens = []
for g0, g1 in zip(idx, idx[1:]):
    t0, t1 = int(rows[g0]["Start_Timestamp"]), int(rows[g1]["Start_Timestamp"])
    busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows[g0:g1])
    gens.append((g0, g1, (t1 - t0) / 1e3, busy / 1e3))
for k, (g0, g1, wall, busy) in enumerate(gens):
    print(f"gen {k:3d}: wall {wall:8.1f} us  busy {busy:8.1f} us  idle {wall - busy:7.1f} us  kernels {g1 - g0}")
if not a.quiet and gens:
    g0, g1, _, _ = gens[a.show]
    t0 = int(rows[g0]["Start_Timestamp"])
    prev = t0
    for r in rows[g0:g1]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        print(f"{(s - t0) / 1e3:8.1f} gap {(s - prev) / 1e3:6.1f} dur {(e - s) / 1e3:6.1f}  {r['Kernel_Name'][:90]}")
        prev = e
