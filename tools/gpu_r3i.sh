# round-3 re-entry check: GPU suite, flagship bench, Ant rollout latency by population
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3i_gpu_suite.log 2>&1 || { tail -40 gpurun_out/r3i_gpu_suite.log; exit 1; }
tail -3 gpurun_out/r3i_gpu_suite.log
timeout -k 10 300 python -u bench.py --steps 50 > gpurun_out/r3i_bench.log 2>&1 || exit 1
tail -1 gpurun_out/r3i_bench.log
timeout -k 10 300 python -u tools/neuro_latency.py 64 1024 8192 > gpurun_out/r3i_neuro_latency.log 2>&1 || exit 1
cat gpurun_out/r3i_neuro_latency.log
timeout -k 10 200 python -u tools/bench_neuro.py --pop 1024 --gens 5 --graph > gpurun_out/r3i_neuro_pop1024.log 2>&1 || exit 1
tail -1 gpurun_out/r3i_neuro_pop1024.log
timeout -k 10 200 python -u tools/bench_neuro.py --pop 1024 --kernel-only > gpurun_out/r3i_neuro_pop1024_ko.log 2>&1 || exit 1
tail -1 gpurun_out/r3i_neuro_pop1024_ko.log
