"""Per-kernel summary of rocprofv3 ``--pmc`` passes (``*counter_collection.csv``).

python tools/pmc_summary.py OUT.txt DIR [DIR ...]   # one DIR per pass, merged by kernel name

For every kernel: dispatches, mean duration, the summed counters of all passes, and the
derived ratios the NOTES "bound by" lines quote:

* ``wait%``    SQ_WAIT_ANY / SQ_WAVE_CYCLES        — waves parked on s_waitcnt / barriers
* ``issue%``   SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES   — waves ready but the pipe was busy
* ``valu%``    SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES
* ``mfma%``    SQ_VALU_MFMA_BUSY_CYCLES / (duration · clock · 1024 SIMDs), clock from
               GRBM_GUI_ACTIVE / 8 / duration when that pass ran (else 2.1 GHz)
* ``ldsc%``    SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
* ``GHz``      GRBM_GUI_ACTIVE / 8 / duration — reads high on dispatches shorter than ≈0.3 ms
               (profiling overhead inside the window), only meaningful for long kernels
* ``HBM GB/s`` (2·FETCH_SIZE + WRITE_SIZE) KiB / duration (gfx950 FETCH_SIZE reads half of a
               wide coalesced stream, /opt/skills/guides/MI355X_MICROARCH.md §rocprofv3)
* ``L2 hit%``  TCC_HIT_sum / (TCC_HIT_sum + TCC_MISS_sum)
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def load(d):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    rows = []
    for f in files:
        with open(f) as fh:
            rows.extend(csv.DictReader(fh))
    return rows


def short(name, grid):
    name = name.replace("(anonymous namespace)::", "")
    if name.startswith("void "):
        name = name[5:]
    name = name.split("(")[0]
    return f"{name[:58]} g{grid}"[:70]


def main():
    out, dirs = sys.argv[1], sys.argv[2:]
    cnt = defaultdict(lambda: defaultdict(float))  # kernel → counter → sum
    disp = defaultdict(set)  # kernel → dispatch ids (per pass)
    dur = defaultdict(list)
    meta = {}
    for p, d in enumerate(dirs):
        for r in load(d):
            k = short(r.get("Kernel_Name", "?"), r.get("Grid_Size", "?"))
            did = (p, r.get("Dispatch_Id"))
            cnt[k][r["Counter_Name"]] += float(r["Counter_Value"])
            if did not in disp[k]:
                disp[k].add(did)
                try:
                    dur[k].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
                except (KeyError, ValueError):
                    pass
                meta[k] = (r.get("VGPR_Count", "?"), r.get("Accum_VGPR_Count", "?"), r.get("LDS_Block_Size", "?"),
                           r.get("Workgroup_Size", "?"), r.get("Grid_Size", "?"))
    npass = max(len(dirs), 1)
    lines = []
    order = sorted(cnt, key=lambda k: -sum(dur[k]))
    hdr = f"{'kernel':70s} {'disp':>5s} {'us':>8s} {'wait%':>6s} {'issue%':>6s} {'valu%':>6s} {'mfma%':>6s} {'ldsc%':>6s} {'HBMGB/s':>8s} {'L2hit%':>6s} {'GHz':>5s}  vgpr/agpr/lds/wg/grid"
    lines.append(hdr)
    for k in order:
        c = cnt[k]
        nd = len(disp[k]) / npass
        us = (sum(dur[k]) / len(dur[k]) / 1e3) if dur[k] else float("nan")
        tot_ns = sum(dur[k]) / npass if dur[k] else float("nan")

        def ratio(a, b, scale=100.0):
            return scale * c[a] / c[b] if c.get(b) else float("nan")

        ghz = c["GRBM_GUI_ACTIVE"] / 8 / tot_ns if c.get("GRBM_GUI_ACTIVE") and tot_ns == tot_ns and tot_ns > 0 else float("nan")
        clk = ghz if ghz == ghz else 2.1
        mfma = 100 * c["SQ_VALU_MFMA_BUSY_CYCLES"] / (tot_ns * clk * 1024) if c.get("SQ_VALU_MFMA_BUSY_CYCLES") and tot_ns > 0 else float("nan")
        hbm = (2 * c.get("FETCH_SIZE", 0) + c.get("WRITE_SIZE", 0)) * 1024 / tot_ns if tot_ns > 0 and ("FETCH_SIZE" in c or "WRITE_SIZE" in c) else float("nan")
        hit = 100 * c["TCC_HIT_sum"] / (c["TCC_HIT_sum"] + c["TCC_MISS_sum"]) if c.get("TCC_HIT_sum", 0) + c.get("TCC_MISS_sum", 0) else float("nan")
        lines.append(f"{k:70s} {nd:5.0f} {us:8.2f} {ratio('SQ_WAIT_ANY', 'SQ_WAVE_CYCLES'):6.1f} {ratio('SQ_WAIT_INST_ANY', 'SQ_WAVE_CYCLES'):6.1f} "
                     f"{ratio('SQ_ACTIVE_INST_VALU', 'SQ_WAVE_CYCLES'):6.1f} {mfma:6.1f} {ratio('SQ_LDS_BANK_CONFLICT', 'SQ_LDS_IDX_ACTIVE'):6.1f} "
                     f"{hbm:8.1f} {hit:6.1f} {ghz:5.2f}  {'/'.join(str(x) for x in meta.get(k, ()))}")
    lines.append("")
    lines.append("raw counter sums (all dispatches of all passes):")
    for k in order[:30]:
        lines.append(f"{k}: " + ", ".join(f"{n}={v:.4g}" for n, v in sorted(cnt[k].items())))
    with open(out, "w") as fh:
        fh.write("\n".join(lines) + "\n")
    print("\n".join(lines[: min(len(lines), 40)]))


if __name__ == "__main__":
    main()
