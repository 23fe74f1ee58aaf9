set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/nsw
for nw in 1 2 1 2; do
  for st in 20 50; do
    NS_WARM=$nw timeout -k 10 200 python -u scratch8/ns1.py --steps $st --warmup 5 > gpurun_out/nsw/b${st}_$nw.log 2>&1 || { tail -5 gpurun_out/nsw/b${st}_$nw.log; exit 1; }
    python -c "import json;d=json.loads(open('gpurun_out/nsw/b${st}_$nw.log').read().strip().splitlines()[-1]);e=d['eigh_stats'];print('ns_warm', $nw, $st, d['ms_per_step'], e['iters_per_gen'], e['schedule_per_gen'], e['capped'], e['fallbacks'], e['recovered'], e['schedule_escalations'], e['max_off_rel'])"
  done
done
NS_WARM=1 timeout -k 10 900 python -u scratch8/ns1.py pytest -q --timeout 600 --timeout-method thread -p no:cacheprovider tests/test_eigh_sbr.py tests/test_sbr_device_gpu.py tests/test_determinism_gpu.py tests/test_distributed_gpu.py > gpurun_out/nsw/t.log 2>&1
rc=$?; tail -2 gpurun_out/nsw/t.log | cut -c1-300; [ $rc -ne 0 ] && grep -m6 "FAILED\|assert" gpurun_out/nsw/t.log | cut -c1-300
exit $rc
