set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/s24
run() {  # label, overrides...
  local lab=$1; shift
  for st in 20 50; do
    timeout -k 10 200 python -u tools/bench_ab.py "$@" -- --steps $st --warmup 5 > gpurun_out/s24/${lab}_${st}.log 2>&1 || { tail -5 gpurun_out/s24/${lab}_${st}.log; return 1; }
    python -c "
import json
d=json.loads(open('gpurun_out/s24/${lab}_${st}.log').read().strip().splitlines()[-1])
e=d.get('eigh_stats',{})
print('$lab', $st, d['ms_per_step'], e.get('iters_per_gen'), e.get('schedule_per_gen'), e.get('schedule_escalations'), e.get('capped'), e.get('lean_guard_stops'), e.get('max_off_rel'))
"
  done
}
run base evoxmi.ops.sbr_device.WARM6_LEAN_FROM=0 || exit 1
run l3d2 evoxmi.ops.sbr_device.WARM6_LEAN_FROM=3 evoxmi.ops.sbr_device.WARM6_DAMP_FROM=2 || exit 1
run l4d2 evoxmi.ops.sbr_device.WARM6_LEAN_FROM=4 evoxmi.ops.sbr_device.WARM6_DAMP_FROM=2 || exit 1
run l3d3 evoxmi.ops.sbr_device.WARM6_LEAN_FROM=3 evoxmi.ops.sbr_device.WARM6_DAMP_FROM=3 || exit 1
