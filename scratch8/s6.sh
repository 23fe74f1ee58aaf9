set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/s6
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -x -p no:cacheprovider tests/test_gemm_blk.py tests/test_kernels_gpu.py -k "blk or h3 or cec2022" > gpurun_out/s6/t1.log 2>&1
rc=$?; tail -3 gpurun_out/s6/t1.log | cut -c1-300; [ $rc -ne 0 ] && { grep -m5 "Error\|assert" gpurun_out/s6/t1.log | cut -c1-300; exit $rc; }
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -x -p no:cacheprovider tests/test_sbr_device_gpu.py tests/test_distributed_gpu.py -k "not 200 and not 600 and not default_lambda" > gpurun_out/s6/t2.log 2>&1
rc=$?; tail -3 gpurun_out/s6/t2.log | cut -c1-300; [ $rc -ne 0 ] && { grep -m5 "Error\|assert" gpurun_out/s6/t2.log | cut -c1-300; exit $rc; }
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > gpurun_out/s6/b20.log 2>&1 && tail -1 gpurun_out/s6/b20.log > gpurun_out/s6/final.jsonl || exit 1
for W in 2 4 8; do
  timeout -k 10 200 python -u bench.py --simulate-rank 0 --world $W --steps 20 --warmup 5 > gpurun_out/s6/sim$W.log 2>&1 && tail -1 gpurun_out/s6/sim$W.log >> gpurun_out/s6/final.jsonl || { tail -5 gpurun_out/s6/sim$W.log; exit 1; }
done
python - <<'PY'
import json
for l in open("gpurun_out/s6/final.jsonl"):
    d = json.loads(l)
    e = d.get("eigh_stats", {})
    print(d["config"]["parallelism"], d["ms_per_step"], (d.get("simulated") or {}).get("projected_ms_with_wire"), e.get("capped"), e.get("max_off_rel"), e.get("schedule_per_gen"), d.get("phases_ms_eager"))
PY
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/s6/kt1 -o kt --output-format csv -- python3 $R/bench.py --steps 40 --warmup 5 --phase-steps 0 > $R/gpurun_out/s6/kt1.log 2>&1 || { tail -20 $R/gpurun_out/s6/kt1.log; exit 1; }
for W in 2 8; do
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/s6/kt$W -o kt --output-format csv -- python3 $R/bench.py --simulate-rank 0 --world $W --steps 40 --warmup 5 --phase-steps 0 > $R/gpurun_out/s6/kt$W.log 2>&1 || { tail -20 $R/gpurun_out/s6/kt$W.log; exit 1; }
done
cd $R
f1=$(find gpurun_out/s6/kt1 -name '*kernel_trace.csv' | head -1)
f2=$(find gpurun_out/s6/kt2 -name '*kernel_trace.csv' | head -1)
f8=$(find gpurun_out/s6/kt8 -name '*kernel_trace.csv' | head -1)
python tools/ktrace_phases.py --gens 20 $f1 $f2 $f8 --labels "1 GPU" "rank 0 of 2 (sim)" "rank 0 of 8 (sim)" > gpurun_out/s6/phases.txt
head -8 gpurun_out/s6/phases.txt
gzip -f $f1 $f2 $f8
