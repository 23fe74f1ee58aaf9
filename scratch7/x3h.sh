set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/s11
J() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);e=d.get('eigh_stats',{});s=d.get('simulated',{});print(sys.argv[2],d['ms_per_step'],d.get('phases_ms_eager'),e.get('max_off_rel'),e.get('fallbacks'),e.get('capped'),e.get('schedule_per_gen'),s.get('projected_ms_with_wire'),s.get('wire_ms_per_gen'))" "$@"; }
for p in x3 x6; do
EVOXMI_SBR_CORR_PREC=$p timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_eigh_sbr.py -k "trajectories" > gpurun_out/s11/parity_$p.log 2>&1; echo "parity $p rc=$?"; grep -o "AssertionError: {.*" gpurun_out/s11/parity_$p.log | head -1
done
for p in x3 x3all x6; do
for st in 20 50; do
EVOXMI_SBR_CORR_PREC=$p timeout -k 10 200 python bench.py --steps $st --warmup 5 > gpurun_out/s11/b${st}_$p.json 2>>gpurun_out/s11/err || { tail gpurun_out/s11/err; exit 1; }
J gpurun_out/s11/b${st}_$p.json "$p b$st"
done
done
timeout -k 10 1000 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu tests/test_gemm_x3.py tests/test_sbr_device_gpu.py tests/test_eigh_sbr.py > gpurun_out/s11/t.log 2>&1 || { tail -30 gpurun_out/s11/t.log; exit 1; }
tail -3 gpurun_out/s11/t.log
