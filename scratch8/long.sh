set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/long2
for f in 1 2 4 6 7 10 12; do
  timeout -k 10 300 python -u bench.py --func $f --steps 1000 --warmup 5 > gpurun_out/long2/f$f.log 2>&1 || { tail -5 gpurun_out/long2/f$f.log; exit 1; }
  python -c "
import json
d=json.loads(open('gpurun_out/long2/f$f.log').read().strip().splitlines()[-1])
e=d.get('eigh_stats',{})
print('F$f', d['ms_per_step'], 'capped', e.get('capped'), 'fallbacks', e.get('fallbacks'), 'max_off_rel', e.get('max_off_rel'), 'mean_iters', e.get('mean_refine_iters'), 'esc', e.get('schedule_escalations'), 'best', d.get('best_fitness'))
"
done
