set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/s30
timeout -k 10 900 python -u -m pytest -q --timeout 400 --timeout-method thread -m gpu tests/ -x -p no:cacheprovider > gpurun_out/s30/full.log 2>&1
rc=$?
tail -15 gpurun_out/s30/full.log | cut -c1-300
[ $rc -ne 0 ] && exit $rc
for st in 20 50; do
timeout -k 10 200 python -u bench.py --steps $st --warmup 5 > gpurun_out/s30/b$st.log 2>&1 && python -c "import json;d=json.loads(open('gpurun_out/s30/b$st.log').read().strip().splitlines()[-1]);e=d['eigh_stats'];print($st, d['ms_per_step'], e['iters_per_gen'], e['schedule_per_gen'], e['capped'], e['max_off_rel'])"
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/s30/kt -o kt --output-format csv -- python3 $R/bench.py --steps 40 --warmup 5 --phase-steps 0 > $R/gpurun_out/s30/kt_bench.log 2>&1 || { cd $R; tail -20 gpurun_out/s30/kt_bench.log; exit 1; }
cd $R
f=$(find gpurun_out/s30/kt -name '*kernel_trace.csv' | head -1)
python tools/ktrace_gen.py $f --marker philox_h --show -2 --agg 20 > gpurun_out/s30/kt_gen.txt
grep "=== last\|eig_out\|sbr_dev_copy" gpurun_out/s30/kt_gen.txt | cut -c1-160 | tail -4
rm -f $f
