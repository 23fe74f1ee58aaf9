# monitor cost by mode, composition functions under graph capture
mkdir -p gpurun_out
set -o pipefail
for m in best device host; do
  timeout -k 10 300 python -u bench.py --monitor $m --phase-steps 0 > gpurun_out/r3ad_bench_mon_$m.log 2>&1 || exit 1
  tail -1 gpurun_out/r3ad_bench_mon_$m.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$m', d['ms_per_step'], d['monitor'])"
done
for f in 9 10 11 12; do
  timeout -k 10 300 python -u bench.py --func $f --steps 30 > gpurun_out/r3ad_bench_f$f.log 2>&1 || exit 1
  tail -1 gpurun_out/r3ad_bench_f$f.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('F$f', d['ms_per_step'], d.get('phases_ms_eager'), d.get('eigh_stats',{}).get('max_off_rel'))"
done
