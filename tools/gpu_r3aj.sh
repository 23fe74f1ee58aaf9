# K6 fused rotation + row-terms epilogue: tests, bench, kernel stats
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_gemm_ks.py tests/test_graph_capture_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "rowterms or gemm or cec" > gpurun_out/r3aj_tests.log 2>&1 || { tail -30 gpurun_out/r3aj_tests.log; exit 1; }
tail -1 gpurun_out/r3aj_tests.log
timeout -k 10 300 python -u bench.py > gpurun_out/r3aj_bench.log 2>&1 || exit 1
tail -1 gpurun_out/r3aj_bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench', d['ms_per_step'], d['eigh_stats'], d.get('phases_ms_eager'))"
timeout -k 10 300 python -u bench.py --func 4 --steps 30 > gpurun_out/r3aj_bench_f4.log 2>&1 || exit 1
tail -1 gpurun_out/r3aj_bench_f4.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('F4', d['ms_per_step'], d.get('phases_ms_eager'))"
