set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/s7
for c in 1 2 3 4 5 6 7 8 0; do
  EVOXMI_H3_CFG=$c timeout -k 10 120 python -u tools/bench_gemm_blk.py --only-h3 --reps 30 --shapes 10000x1000x1000,5000x1000x1000,2500x1000x1000,1250x1000x1000 >> gpurun_out/s7/sweep.jsonl 2>gpurun_out/s7/err$c.log || { tail -5 gpurun_out/s7/err$c.log; exit 1; }
done
python - <<'PY'
import json, collections
t = collections.defaultdict(dict)
for l in open("gpurun_out/s7/sweep.jsonl"):
    d = json.loads(l); t[d["shape"]][d["h3_cfg"]] = d["h3_gemm_us"]
for sh, r in t.items():
    print(sh, " ".join(f"{k}:{v}" for k, v in sorted(r.items())))
PY
