set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/s9
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread -x -p no:cacheprovider tests/test_eigh_sbr.py -k "sbr16_kernels" > gpurun_out/s9/t0.log 2>&1
rc=$?; tail -3 gpurun_out/s9/t0.log | cut -c1-300; [ $rc -ne 0 ] && { grep -m8 "Error\|assert" gpurun_out/s9/t0.log | cut -c1-300; exit $rc; }
for v in 1 0; do
  EVOXMI_SBR_BLOCK_1W=$v timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --phase-steps 0 > gpurun_out/s9/b20_$v.log 2>&1 || { tail -5 gpurun_out/s9/b20_$v.log; exit 1; }
  EVOXMI_SBR_BLOCK_1W=$v timeout -k 10 200 python -u bench.py --steps 50 --warmup 5 > gpurun_out/s9/b50_$v.log 2>&1 || { tail -5 gpurun_out/s9/b50_$v.log; exit 1; }
  for st in 20 50; do python -c "import json;d=json.loads(open('gpurun_out/s9/b${st}_$v.log').read().strip().splitlines()[-1]);e=d['eigh_stats'];print('1w=$v', $st, d['ms_per_step'], e['iters_per_gen'], e['schedule_per_gen'], e['capped'], e['max_off_rel'], d.get('phases_ms_eager'))"; done
done
timeout -k 10 900 python -u -m pytest -q --timeout 400 --timeout-method thread -x -p no:cacheprovider tests/test_eigh_sbr.py tests/test_sbr_device_gpu.py tests/test_determinism_gpu.py tests/test_distributed_gpu.py > gpurun_out/s9/t1.log 2>&1
rc=$?; tail -3 gpurun_out/s9/t1.log | cut -c1-300; [ $rc -ne 0 ] && { grep -m8 "Error\|assert\|FAILED" gpurun_out/s9/t1.log | cut -c1-300; exit $rc; }
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/s9/kt1 -o kt --output-format csv -- python3 $R/bench.py --steps 40 --warmup 5 --phase-steps 0 > $R/gpurun_out/s9/kt1.log 2>&1 || { tail -20 $R/gpurun_out/s9/kt1.log; exit 1; }
cd $R
f1=$(find gpurun_out/s9/kt1 -name '*kernel_trace.csv' | head -1)
python tools/ktrace_gen.py $f1 --marker philox_h --show -2 --agg 20 > gpurun_out/s9/kt_gen1.txt
grep "=== last\|block1w\|block_kernel" gpurun_out/s9/kt_gen1.txt | tail -4 | cut -c1-150
gzip -f $f1
