mkdir -p gpurun_out
set -o pipefail
timeout -k 10 120 python -u tools/bench_sort.py > gpurun_out/r3_sort_microbench.log 2>&1 || exit 1
cat gpurun_out/r3_sort_microbench.log
timeout -k 10 300 python -u bench.py > gpurun_out/r3h_bench.log 2>&1 || exit 1
tail -1 gpurun_out/r3h_bench.log
bash tools/gpu_pmc.sh
