"""Summarise a rocprofv3 kernel_stats.csv as µs per generation."""
import csv
import sys

path, gens = sys.argv[1], float(sys.argv[2])
rows = list(csv.DictReader(open(path)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total kernel time {tot / 1e6:.2f} ms, per gen {tot / 1e3 / gens:.1f} us")
for r in rows[: int(sys.argv[3]) if len(sys.argv) > 3 else 25]:
    print(f"{float(r['TotalDurationNs']) / 1e3 / gens:9.1f} us/gen  calls/gen {int(r['Calls']) / gens:7.1f}  avg {float(r['AverageNs']) / 1000:8.2f}us  {r['Name'][:100]}")
