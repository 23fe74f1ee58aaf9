set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/s7
timeout -k 10 120 python tools/bench_gemm_x3.py > gpurun_out/s7/x3_gemm.jsonl 2>gpurun_out/s7/x3.err || { tail gpurun_out/s7/x3.err; exit 1; }
cat gpurun_out/s7/x3_gemm.jsonl
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gemm_x3.py tests/test_gemm_blk.py > gpurun_out/s7/x3_t.log 2>&1 || { tail -30 gpurun_out/s7/x3_t.log; exit 1; }
tail -1 gpurun_out/s7/x3_t.log
for p in x6 x3; do
EVOXMI_SBR_CORR_PREC=$p timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/s7/x3_b20_$p.json 2>>gpurun_out/s7/x3.err || { tail gpurun_out/s7/x3.err; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/s7/x3_b20_$p.json').read().strip().splitlines()[-1]);e=d['eigh_stats'];print('$p b20',d['ms_per_step'],d['phases_ms_eager'],e['max_off_rel'],e['fallbacks'],e['capped'],e['iters_per_gen'],e['schedule_per_gen'])"
EVOXMI_SBR_CORR_PREC=$p timeout -k 10 200 python bench.py --steps 50 --warmup 5 > gpurun_out/s7/x3_b50_$p.json 2>>gpurun_out/s7/x3.err || { tail gpurun_out/s7/x3.err; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/s7/x3_b50_$p.json').read().strip().splitlines()[-1]);e=d['eigh_stats'];print('$p b50',d['ms_per_step'],d['phases_ms_eager'],e['max_off_rel'],e['fallbacks'],e['capped'],e['iters_per_gen'],e['schedule_per_gen'])"
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/s7/kt -o kt --output-format csv -- python3 $R/bench.py --steps 40 --warmup 5 --phase-steps 0 > $R/gpurun_out/s7/kt_bench.log 2>&1 || { cd $R; tail -20 gpurun_out/s7/kt_bench.log; exit 1; }
cd $R
f=$(find gpurun_out/s7/kt -name '*kernel_trace.csv' | head -1)
python tools/ktrace_gen.py $f --marker philox_h --show -2 --agg 20 > gpurun_out/s7/kt_gen_x3.txt
grep -A30 "=== last" gpurun_out/s7/kt_gen_x3.txt | cut -c1-160
rm -f $f
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_sbr_device_gpu.py tests/test_eigh_sbr.py > gpurun_out/s7/x3_sbr_t.log 2>&1 || { tail -30 gpurun_out/s7/x3_sbr_t.log; exit 1; }
tail -3 gpurun_out/s7/x3_sbr_t.log
