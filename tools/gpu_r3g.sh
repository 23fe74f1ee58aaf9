mkdir -p gpurun_out
set -o pipefail
timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -q --timeout 100 --timeout-method thread -m gpu -k "argsort" > gpurun_out/r3g_sort_tests.log 2>&1 || { tail -30 gpurun_out/r3g_sort_tests.log; exit 1; }
tail -2 gpurun_out/r3g_sort_tests.log
timeout -k 10 120 python -u tools/bench_sort.py > gpurun_out/r3_sort_microbench.log 2>&1 || exit 1
cat gpurun_out/r3_sort_microbench.log
