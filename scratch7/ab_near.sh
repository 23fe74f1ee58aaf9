set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/s25
run() {  # label, overrides...
  local lab=$1; shift
  for st in 20 50; do
    timeout -k 10 200 python -u tools/bench_ab.py "$@" -- --steps $st --warmup 5 > gpurun_out/s25/${lab}_${st}.log 2>&1 || { tail -5 gpurun_out/s25/${lab}_${st}.log; return 1; }
    python -c "
import json
d=json.loads(open('gpurun_out/s25/${lab}_${st}.log').read().strip().splitlines()[-1])
e=d.get('eigh_stats',{})
print('$lab', $st, d['ms_per_step'], e.get('iters_per_gen'), e.get('schedule_per_gen'), e.get('schedule_escalations'), e.get('capped'), e.get('max_off_rel'))
"
  done
}
CFG="{'theta0': 1.0, 'theta_kappa': 0.05, 'thr_fac': 0.3, 'block_sweeps': 2, 'damp_tau': 1.0, 'damp_kappa': 1.0, 'ns_kappa': 0.3, 'ns_iters': 2"
run base "evoxmi.ops.sbr_device.DEVICE_CFG=$CFG, 'near_only': 1.5}" || exit 1
run n3 "evoxmi.ops.sbr_device.DEVICE_CFG=$CFG, 'near_only': 3.0}" || exit 1
run n4 "evoxmi.ops.sbr_device.DEVICE_CFG=$CFG, 'near_only': 4.0}" || exit 1
run n6 "evoxmi.ops.sbr_device.DEVICE_CFG=$CFG, 'near_only': 6.0}" || exit 1
