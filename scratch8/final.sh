set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/final
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1 || { tail -20 gpurun_out/final/smoke.log; exit 1; }
tail -1 gpurun_out/final/smoke.log
timeout -k 10 200 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/final/b20.log 2>&1 && tail -1 gpurun_out/final/b20.log > gpurun_out/final/final.jsonl || { tail -5 gpurun_out/final/b20.log; exit 1; }
timeout -k 10 200 python -u bench.py --steps 50 --warmup 5 > gpurun_out/final/b50.log 2>&1 && tail -1 gpurun_out/final/b50.log >> gpurun_out/final/final.jsonl || { tail -5 gpurun_out/final/b50.log; exit 1; }
for W in 2 4 8; do
  timeout -k 10 200 python -u bench.py --simulate-rank 0 --world $W --steps 20 --warmup 5 > gpurun_out/final/sim$W.log 2>&1 && tail -1 gpurun_out/final/sim$W.log >> gpurun_out/final/final.jsonl || { tail -5 gpurun_out/final/sim$W.log; exit 1; }
done
python - <<'PY'
import json
for l in open("gpurun_out/final/final.jsonl"):
    d = json.loads(l)
    e = d.get("eigh_stats", {})
    print(d["config"]["parallelism"], d["steps"], d["ms_per_step"], (d.get("simulated") or {}).get("projected_ms_with_wire"), e.get("capped"), e.get("max_off_rel"), e.get("schedule_per_gen"), d.get("gemm_precision"))
PY
timeout -k 10 1500 python -u -m pytest -q --timeout 400 --timeout-method thread -m gpu tests/ -p no:cacheprovider > gpurun_out/final/full.log 2>&1
rc=$?
tail -4 gpurun_out/final/full.log | cut -c1-300
[ $rc -ne 0 ] && grep "FAILED" gpurun_out/final/full.log | head
exit $rc
