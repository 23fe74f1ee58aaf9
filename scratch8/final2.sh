set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/final2
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final2/smoke.log 2>&1 || { tail -20 gpurun_out/final2/smoke.log; exit 1; }
tail -1 gpurun_out/final2/smoke.log
timeout -k 10 200 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/final2/b20.log 2>&1 && tail -1 gpurun_out/final2/b20.log > gpurun_out/final2/final.jsonl || { tail -5 gpurun_out/final2/b20.log; exit 1; }
timeout -k 10 200 python -u bench.py --steps 50 --warmup 5 > gpurun_out/final2/b50.log 2>&1 && tail -1 gpurun_out/final2/b50.log >> gpurun_out/final2/final.jsonl || { tail -5 gpurun_out/final2/b50.log; exit 1; }
for f in 1 2 4 6 7 10 12; do
  timeout -k 10 300 python -u bench.py --func $f --steps 1000 --warmup 5 > gpurun_out/final2/f$f.log 2>&1 && tail -1 gpurun_out/final2/f$f.log >> gpurun_out/final2/long.jsonl || { tail -5 gpurun_out/final2/f$f.log; exit 1; }
done
python - <<'PY'
import json
for fn in ("gpurun_out/final2/final.jsonl", "gpurun_out/final2/long.jsonl"):
    for l in open(fn):
        d = json.loads(l); e = d.get("eigh_stats", {})
        print(d["config"]["model"][-30:], d["steps"], d["ms_per_step"], e.get("capped"), e.get("fallbacks"), e.get("max_off_rel"), e.get("mean_refine_iters"), e.get("schedule_escalations"), (e.get("schedule_per_gen") or "")[:24])
PY
timeout -k 10 1500 python -u -m pytest -q --timeout 400 --timeout-method thread -m gpu tests/ -p no:cacheprovider > gpurun_out/final2/full.log 2>&1
rc=$?
tail -2 gpurun_out/final2/full.log | cut -c1-300
[ $rc -ne 0 ] && grep "FAILED" gpurun_out/final2/full.log | head
exit $rc
