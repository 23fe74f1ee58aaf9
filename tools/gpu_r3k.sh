# articulated Ant after the force/wrench simplification, no-SLP build at 2 waves / SIMD
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_determinism_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "ant" > gpurun_out/r3k_ant_tests.log 2>&1 || { tail -40 gpurun_out/r3k_ant_tests.log; exit 1; }
tail -2 gpurun_out/r3k_ant_tests.log
timeout -k 10 200 python -u tools/neuro_latency.py 64 1024 8192 > gpurun_out/r3k_neuro_latency.log 2>&1 || exit 1
cat gpurun_out/r3k_neuro_latency.log
timeout -k 10 200 python -u tools/bench_neuro.py --pop 1024 --gens 5 --graph > gpurun_out/r3k_neuro_pop1024.log 2>&1 || exit 1
tail -1 gpurun_out/r3k_neuro_pop1024.log
timeout -k 10 300 python -u tools/bench_neuro.py --pop 8192 --gens 5 --graph > gpurun_out/r3k_neuro_pop8192.log 2>&1 || exit 1
tail -1 gpurun_out/r3k_neuro_pop8192.log
