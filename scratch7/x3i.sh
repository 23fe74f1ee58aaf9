set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/s12
J() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);e=d.get('eigh_stats',{});s=d.get('simulated',{});print(sys.argv[2],d['ms_per_step'],d.get('phases_ms_eager'),e.get('max_off_rel'),e.get('fallbacks'),e.get('capped'),e.get('schedule_per_gen'),s.get('projected_ms_with_wire'),s.get('wire_ms_per_gen'))" "$@"; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s12/smoke.log 2>&1 || { tail gpurun_out/s12/smoke.log; exit 1; }
tail -1 gpurun_out/s12/smoke.log
for st in 20 50; do
timeout -k 10 200 python bench.py --steps $st --warmup 5 > gpurun_out/s12/b$st.json 2>>gpurun_out/s12/err || { tail gpurun_out/s12/err; exit 1; }
J gpurun_out/s12/b$st.json "b$st"
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/s12/kt -o kt --output-format csv -- python3 $R/bench.py --steps 40 --warmup 5 --phase-steps 0 > $R/gpurun_out/s12/kt_bench.log 2>&1 || { cd $R; tail -20 gpurun_out/s12/kt_bench.log; exit 1; }
cd $R
f=$(find gpurun_out/s12/kt -name '*kernel_trace.csv' | head -1)
python tools/ktrace_gen.py $f --marker philox_h --show -2 --agg 20 > gpurun_out/s12/kt_gen.txt
grep -A6 "=== last" gpurun_out/s12/kt_gen.txt | cut -c1-160
rm -f $f
timeout -k 10 1100 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu tests/test_sbr_device_gpu.py tests/test_eigh_sbr.py tests/test_distributed_gpu.py tests/test_graph_capture_gpu.py tests/test_determinism_gpu.py > gpurun_out/s12/t.log 2>&1 || { tail -30 gpurun_out/s12/t.log; exit 1; }
tail -3 gpurun_out/s12/t.log
