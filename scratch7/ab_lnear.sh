set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/s26
run() {  # label, overrides...
  local lab=$1; shift
  for st in 20 50; do
    timeout -k 10 200 python -u tools/bench_ab.py "$@" -- --steps $st --warmup 5 > gpurun_out/s26/${lab}_${st}.log 2>&1 || { tail -5 gpurun_out/s26/${lab}_${st}.log; return 1; }
    python -c "
import json
d=json.loads(open('gpurun_out/s26/${lab}_${st}.log').read().strip().splitlines()[-1])
e=d.get('eigh_stats',{})
print('$lab', $st, d['ms_per_step'], e.get('iters_per_gen'), e.get('schedule_per_gen'), e.get('schedule_escalations'), e.get('capped'), e.get('max_off_rel'))
"
  done
}
run base evoxmi.ops.sbr_device.LATE_NEAR_ONLY=None || exit 1
run ln3 evoxmi.ops.sbr_device.LATE_NEAR_ONLY=3.0 || exit 1
run ln4 evoxmi.ops.sbr_device.LATE_NEAR_ONLY=4.0 || exit 1
