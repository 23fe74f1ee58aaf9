set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/s8
J() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);e=d.get('eigh_stats',{});s=d.get('simulated',{});print(sys.argv[2],d['ms_per_step'],d.get('phases_ms_eager'),e.get('max_off_rel'),e.get('fallbacks'),e.get('capped'),e.get('schedule_per_gen'),s.get('projected_ms_with_wire'),s.get('wire_ms_per_gen'))" "$@"; }
for st in 20 50; do
timeout -k 10 200 python bench.py --steps $st --warmup 5 > gpurun_out/s8/b${st}_o2.json 2>>gpurun_out/s8/err || { tail gpurun_out/s8/err; exit 1; }
J gpurun_out/s8/b${st}_o2.json "order2 b$st"
timeout -k 10 200 python tools/bench_ab.py evoxmi.ops.sbr_device.ORDER2_THR=0 -- --steps $st --warmup 5 > gpurun_out/s8/b${st}_noo2.json 2>>gpurun_out/s8/err || { tail gpurun_out/s8/err; exit 1; }
J gpurun_out/s8/b${st}_noo2.json "no-order2 b$st"
done
timeout -k 10 200 python tools/bench_mo.py --algo moead > gpurun_out/s8/moead_1.json 2>>gpurun_out/s8/err || { tail gpurun_out/s8/err; exit 1; }
tail -1 gpurun_out/s8/moead_1.json | cut -c1-300
for w in 2 8; do
timeout -k 10 200 python tools/bench_mo.py --algo moead --simulate-rank 0 --world $w > gpurun_out/s8/moead_sim$w.json 2>>gpurun_out/s8/err || { tail gpurun_out/s8/err; exit 1; }
tail -1 gpurun_out/s8/moead_sim$w.json | cut -c1-400
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/s8/kt -o kt --output-format csv -- python3 $R/bench.py --steps 40 --warmup 5 --phase-steps 0 > $R/gpurun_out/s8/kt_bench.log 2>&1 || { cd $R; tail -20 gpurun_out/s8/kt_bench.log; exit 1; }
cd $R
f=$(find gpurun_out/s8/kt -name '*kernel_trace.csv' | head -1)
python tools/ktrace_gen.py $f --marker philox_h --show -2 --agg 20 > gpurun_out/s8/kt_gen.txt
grep -A32 "=== last" gpurun_out/s8/kt_gen.txt | cut -c1-160
rm -f $f
timeout -k 10 1000 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gemm_x3.py tests/test_gemm_blk.py tests/test_sbr_device_gpu.py tests/test_eigh_sbr.py tests/test_distributed_gpu.py tests/test_moead_sharded.py > gpurun_out/s8/t.log 2>&1 || { tail -30 gpurun_out/s8/t.log; exit 1; }
tail -3 gpurun_out/s8/t.log
