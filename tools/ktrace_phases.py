"""Per-phase kernel time of the flagship generation from rocprofv3 kernel traces.

Compares runs (e.g. one GPU against ``bench.py --simulate-rank 0 --world 8``) over their
last N generations.  Generations are cut at the generation's key split (``philox_words``,
the last kernel of every generation on both paths: the sharded ask samples its 1/N rows with
other kernels than the one-GPU ask).  Inside a generation:

* eigh      — after ``cov_pad`` (the covariance update) up to ``eig_out``: the replicated,
              device-controlled eigensolve
* sharded   — everything else: sampling, evaluation, ranking / selection, centring, the
              rank-μ GEMM, paths, ``cov_pad``, the C^-1/2 product and bookkeeping (and,
              simulated, the same-size local stand-ins of the collectives)

and a per-kernel table of the non-eigh kernels (µs per generation in each trace).

    python tools/ktrace_phases.py --gens 20 one_gpu.csv sim8.csv [--labels "1 GPU" "rank 0 of 8"]
"""
import argparse
import csv
import gzip

PHASES = ("sharded", "eigh")


def generations(path, marker):
    f = gzip.open(path, "rt") if path.endswith(".gz") else open(path)
    rows = sorted(csv.DictReader(f), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
    return [rows[a:b] for a, b in zip(idx, idx[1:])]


def classify(gen):
    out = {p: 0.0 for p in PHASES}
    per = {}
    stage = "pre"
    for r in gen:
        name = r["Kernel_Name"]
        dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        ph = "eigh" if stage == "eigh" else "sharded"
        if stage == "pre" and "cov_pad" in name:
            stage = "eigh"
        elif stage == "eigh" and "eig_out" in name:
            stage = "post"
        out[ph] += dur
        if ph == "sharded":
            short = name.replace("(anonymous namespace)::", "").replace("void ", "")
            short = short.split("(")[0][:70]
            per[short] = per.get(short, 0.0) + dur
    wall = (int(gen[-1]["End_Timestamp"]) - int(gen[0]["Start_Timestamp"])) / 1e3
    return out, wall, len(gen), per


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("traces", nargs="+")
    ap.add_argument("--labels", nargs="*")
    ap.add_argument("--gens", type=int, default=20)
    ap.add_argument("--marker", default="philox_words")
    a = ap.parse_args()
    labels = a.labels or a.traces
    res, pers = [], []
    for t in a.traces:
        gens = generations(t, a.marker)[-a.gens:]
        acc = {p: 0.0 for p in PHASES}
        wall = kern = 0.0
        per = {}
        for g in gens:
            ph, w, k, pk = classify(g)
            for p in PHASES:
                acc[p] += ph[p] / len(gens)
            for n, v in pk.items():
                per[n] = per.get(n, 0.0) + v / len(gens)
            wall += w / len(gens)
            kern += k / len(gens)
        res.append((acc, wall, kern, len(gens)))
        pers.append(per)
    head = "| phase (µs / generation, kernel busy) | " + " | ".join(labels) + (" | ratio |" if len(res) == 2 else " |")
    print(head)
    print("|" + "---|" * (len(res) + 1 + (len(res) == 2)))
    for p in PHASES + ("all",):
        vals = []
        for acc, _, _, _ in res:
            if p == "all":
                vals.append(sum(acc.values()))
            else:
                vals.append(acc[p])
        ratio = f" {vals[1] / vals[0]:.2f} |" if len(res) == 2 and vals[0] > 0 else ""
        print(f"| {p} | " + " | ".join(f"{v:.1f}" for v in vals) + " |" + ratio)
    print("| wall (first kernel start → last kernel end) | " + " | ".join(f"{w:.1f}" for _, w, _, _ in res) + " |" +
          (" |" if len(res) == 2 else ""))
    print("| kernels / generation | " + " | ".join(f"{k:.0f}" for _, _, k, _ in res) + " |" + (" |" if len(res) == 2 else ""))
    print(f"\n(last {res[0][3]} generations of each trace)\n")
    print("| non-eigh kernel (µs / generation) | " + " | ".join(labels) + " |")
    print("|" + "---|" * (len(res) + 1))
    names = sorted(set().union(*pers), key=lambda n: -max(p.get(n, 0.0) for p in pers))
    for n in names:
        print(f"| `{n}` | " + " | ".join(f"{p.get(n, 0.0):.1f}" for p in pers) + " |")


if __name__ == "__main__":
    main()
