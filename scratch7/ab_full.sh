set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/s20
for fs in 5 4 3; do
  for st in 20 50; do
    timeout -k 10 200 python -u tools/bench_ab.py evoxmi.ops.sbr_device.FULL_SLOTS=$fs -- --steps $st --warmup 5 > gpurun_out/s20/fs${fs}_${st}.log 2>&1 || { tail -5 gpurun_out/s20/fs${fs}_${st}.log; exit 1; }
    python -c "
import json,sys
d=json.loads(open('gpurun_out/s20/fs${fs}_${st}.log').read().strip().splitlines()[-1])
print('FULL_SLOTS=$fs steps=$st', d['ms_per_step'], d.get('schedule_per_gen'), d.get('schedule_escalations'), {k:v for k,v in d.get('eigh_stats',{}).items() if k in ('capped','fallbacks','max_off_rel','iters_per_gen')})
"
  done
done
