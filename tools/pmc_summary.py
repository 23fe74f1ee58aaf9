"""Aggregate rocprofv3 counter_collection.csv per kernel (mean over dispatches)."""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
agg = defaultdict(lambda: defaultdict(list))
meta = {}
for r in rows:
    name = r["Kernel_Name"]
    if "(anonymous namespace)::" in name[:40]:
        short = name[:110]
    else:
        short = name.split("(")[0][-70:] or name[:110]
    key = short + f" [vgpr={r['VGPR_Count']} agpr={r['Accum_VGPR_Count']} lds={r['LDS_Block_Size']}]"
    agg[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
    meta[key] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
filt = sys.argv[2] if len(sys.argv) > 2 else ""
for k, cs in agg.items():
    if filt and filt not in k:
        continue
    m = {c: sum(v) / len(v) for c, v in cs.items()}
    line = f"{k}\n   dur~{meta[k]:.1f}us " + " ".join(f"{c}={v:.3g}" for c, v in sorted(m.items()))
    if "SQ_WAVE_CYCLES" in m and m["SQ_WAVE_CYCLES"]:
        w = m["SQ_WAVE_CYCLES"]
        line += f"\n   wait_any={m.get('SQ_WAIT_ANY', 0) / w:.2f} wait_inst={m.get('SQ_WAIT_INST_ANY', 0) / w:.2f} active={m.get('SQ_ACTIVE_INST_ANY', 0) / w:.2f}"
    if "SQ_VALU_MFMA_BUSY_CYCLES" in m and "SQ_BUSY_CYCLES" in m and m["SQ_BUSY_CYCLES"]:
        line += f" mfma_busy/busy={m['SQ_VALU_MFMA_BUSY_CYCLES'] / m['SQ_BUSY_CYCLES']:.2f}"
    print(line)
