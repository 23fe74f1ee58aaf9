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
ap.add_argument("--agg", type=int, default=0)
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

# --agg N: per-kernel totals over the last N full generations (µs per generation)
import sys as _sys

if "--agg" in _sys.argv:
    n = int(_sys.argv[_sys.argv.index("--agg") + 1])
    sel = gens[-n:]
    agg = {}
    for g0, g1, _, _ in sel:
        for r in rows[g0:g1]:
            nm = r["Kernel_Name"][:110]
            d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            c, t = agg.get(nm, (0, 0.0))
            agg[nm] = (c + 1, t + d)
    walls = sum(g[2] for g in sel) / len(sel)
    busy = sum(g[3] for g in sel) / len(sel)
    print(f"=== last {len(sel)} generations: wall {walls:.1f} us, busy {busy:.1f} us per generation")
    for nm, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print(f"{t / len(sel):9.1f} us/gen  calls/gen {c / len(sel):5.1f}  avg {t / c:7.2f} us  {nm}")
