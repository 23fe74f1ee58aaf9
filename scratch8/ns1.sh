set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/ns1
for ns in 1 2; do
  for st in 20 50; do
    NS_LATE=$ns timeout -k 10 200 python -u scratch8/ns1.py --steps $st --warmup 5 --phase-steps 0 > gpurun_out/ns1/b${st}_$ns.log 2>&1 || { tail -5 gpurun_out/ns1/b${st}_$ns.log; exit 1; }
    python -c "import json;d=json.loads(open('gpurun_out/ns1/b${st}_$ns.log').read().strip().splitlines()[-1]);e=d['eigh_stats'];print('ns', $ns, $st, d['ms_per_step'], e['iters_per_gen'], e['schedule_per_gen'], e['capped'], e['max_off_rel'])"
  done
done
NS_LATE=1 timeout -k 10 900 python -u scratch8/ns1.py pytest -q --timeout 600 --timeout-method thread -p no:cacheprovider tests/test_eigh_sbr.py::test_cmaes_trajectories_sbr_vs_library_eigh tests/test_sbr_device_gpu.py > gpurun_out/ns1/t.log 2>&1
rc=$?; tail -3 gpurun_out/ns1/t.log | cut -c1-300; [ $rc -ne 0 ] && grep -m6 "FAILED\|assert" gpurun_out/ns1/t.log | cut -c1-300
exit $rc
