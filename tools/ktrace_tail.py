"""Kernel sequence of the last generation in a rocprofv3 kernel_trace.csv (eager run):
the trace is cut at the last occurrence of a marker kernel (default: philox_fill)."""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
marker = sys.argv[2] if len(sys.argv) > 2 else "philox_fill"
idx = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
start = idx[-2] if len(idx) >= 2 else 0
end = idx[-1]
tot = 0
for r in rows[start:end]:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    tot += d
    print(f"{d:9.2f} us  {r['Kernel_Name'][:140]}")
print(f"{end - start} kernels, {tot:.1f} us")
