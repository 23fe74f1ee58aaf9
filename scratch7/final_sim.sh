set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/s21
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > gpurun_out/s21/b20.log 2>&1 && tail -1 gpurun_out/s21/b20.log > gpurun_out/s21/final.jsonl
timeout -k 10 200 python -u bench.py --steps 50 --warmup 5 > gpurun_out/s21/b50.log 2>&1 && tail -1 gpurun_out/s21/b50.log >> gpurun_out/s21/final.jsonl
for W in 2 4 8; do
  timeout -k 10 200 python -u bench.py --simulate-rank 0 --world $W --steps 20 --warmup 5 > gpurun_out/s21/sim$W.log 2>&1 && tail -1 gpurun_out/s21/sim$W.log >> gpurun_out/s21/final.jsonl || { tail -5 gpurun_out/s21/sim$W.log; exit 1; }
done
python - <<'PY'
import json
for l in open("gpurun_out/s21/final.jsonl"):
    d = json.loads(l)
    print(d.get("n_gpus"), d.get("steps"), d["ms_per_step"], d["config"]["parallelism"], (d.get("simulated") or {}).get("projected_ms_with_wire"), d.get("eigh_stats", {}).get("capped"), d.get("eigh_stats", {}).get("max_off_rel"))
PY
