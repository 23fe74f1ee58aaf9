set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/s2
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -x -p no:cacheprovider tests/test_eigh_sbr.py tests/test_sbr_device_gpu.py -k "not 200 and not 600 and not default_lambda" > gpurun_out/s2/t.log 2>&1
rc=$?; tail -4 gpurun_out/s2/t.log | cut -c1-300; [ $rc -ne 0 ] && exit $rc
for st in 20 50; do
timeout -k 10 200 python -u bench.py --steps $st --warmup 5 > gpurun_out/s2/b$st.log 2>&1 && python -c "import json;d=json.loads(open('gpurun_out/s2/b$st.log').read().strip().splitlines()[-1]);e=d['eigh_stats'];print($st, d['ms_per_step'], e['iters_per_gen'], e['schedule_per_gen'], e['capped'], e['max_off_rel'], d['phases_ms_eager'])" || exit 1
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/s2/kt1 -o kt --output-format csv -- python3 $R/bench.py --steps 40 --warmup 5 --phase-steps 0 > $R/gpurun_out/s2/kt1.log 2>&1 || { tail -20 $R/gpurun_out/s2/kt1.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/s2/kt8 -o kt --output-format csv -- python3 $R/bench.py --simulate-rank 0 --world 8 --steps 40 --warmup 5 --phase-steps 0 > $R/gpurun_out/s2/kt8.log 2>&1 || { tail -20 $R/gpurun_out/s2/kt8.log; exit 1; }
cd $R
f1=$(find gpurun_out/s2/kt1 -name '*kernel_trace.csv' | head -1)
f8=$(find gpurun_out/s2/kt8 -name '*kernel_trace.csv' | head -1)
python tools/ktrace_phases.py --gens 20 $f1 $f8 --labels "1 GPU" "rank 0 of 8 (simulated)" > gpurun_out/s2/phases.txt
python tools/ktrace_gen.py $f1 --marker philox_h --show -2 --agg 20 > gpurun_out/s2/kt_gen1.txt
python tools/ktrace_gen.py $f8 --marker philox_h --show -2 --agg 20 > gpurun_out/s2/kt_gen8.txt
cat gpurun_out/s2/phases.txt
grep sbr16_block gpurun_out/s2/kt_gen1.txt | tail -2 | cut -c1-120
tail -1 gpurun_out/s2/kt1.log | cut -c1-200; tail -1 gpurun_out/s2/kt8.log | cut -c1-200
rm -f $f1 $f8
