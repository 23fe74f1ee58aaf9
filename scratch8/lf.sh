set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/lf
for lf in 2 3 2 3; do
  for st in 50; do
    LATE_FULL=$lf timeout -k 10 200 python -u scratch8/ns1.py --steps $st --warmup 5 > gpurun_out/lf/b${st}_$lf.log 2>&1 || { tail -5 gpurun_out/lf/b${st}_$lf.log; exit 1; }
    python -c "import json;d=json.loads(open('gpurun_out/lf/b${st}_$lf.log').read().strip().splitlines()[-1]);e=d['eigh_stats'];print('late_full', $lf, $st, d['ms_per_step'], e['iters_per_gen'], e['schedule_per_gen'], e['capped'], e['lean_guard_stops'], e['schedule_escalations'], e['max_off_rel'])"
  done
done
for f in 1 12; do
  LATE_FULL=2 timeout -k 10 300 python -u scratch8/ns1.py --func $f --steps 1000 --warmup 5 > gpurun_out/lf/f$f.log 2>&1 || { tail -5 gpurun_out/lf/f$f.log; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/lf/f$f.log').read().strip().splitlines()[-1]);e=d['eigh_stats'];print('F$f late_full 2', d['ms_per_step'], e['capped'], e['lean_guard_stops'], e['schedule_escalations'], e['max_off_rel'], e['mean_refine_iters'])"
done
