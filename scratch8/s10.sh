set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/s10
for v in x3late x3; do
  for st in 20 50; do
  EVOXMI_SBR_CORR_PREC=$v timeout -k 10 200 python -u bench.py --steps $st --warmup 5 --phase-steps 0 > gpurun_out/s10/b${st}_$v.log 2>&1 || { tail -5 gpurun_out/s10/b${st}_$v.log; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/s10/b${st}_$v.log').read().strip().splitlines()[-1]);e=d['eigh_stats'];print('$v', $st, d['ms_per_step'], e['iters_per_gen'], e['schedule_per_gen'], e['capped'], e['max_off_rel'])"
  done
done
EVOXMI_SBR_CORR_PREC=x3late timeout -k 10 1100 python -u -m pytest -q --timeout 500 --timeout-method thread -p no:cacheprovider tests/test_eigh_sbr.py tests/test_sbr_device_gpu.py tests/test_determinism_gpu.py tests/test_cmaes_schedule.py > gpurun_out/s10/t.log 2>&1
rc=$?; tail -4 gpurun_out/s10/t.log | cut -c1-300; [ $rc -ne 0 ] && { grep "FAILED\|Error" gpurun_out/s10/t.log | head -8 | cut -c1-300; }
exit $rc
