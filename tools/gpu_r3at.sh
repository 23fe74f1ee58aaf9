# K19: two-pass merge argsort (chunk rank + co-rank merge) tests and microbench
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "argsort" > gpurun_out/r3at_sort_tests.log 2>&1 || { tail -40 gpurun_out/r3at_sort_tests.log; exit 1; }
tail -2 gpurun_out/r3at_sort_tests.log
timeout -k 10 200 python -u tools/bench_sort.py > gpurun_out/r3at_sort_bench.log 2>&1 || exit 1
cat gpurun_out/r3at_sort_bench.log
