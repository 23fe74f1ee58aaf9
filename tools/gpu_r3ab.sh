# Ant rollout with 4-wave workgroups: placement trace, tests, OpenES pop 1024 / 8192
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_determinism_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "ant" > gpurun_out/r3ab_ant_tests.log 2>&1 || { tail -40 gpurun_out/r3ab_ant_tests.log; exit 1; }
tail -1 gpurun_out/r3ab_ant_tests.log
timeout -k 10 100 python -u tools/bench_neuro.py --pop 1024 --gens 6 --dump-pop /tmp/pop6.pt > /dev/null 2>&1 || exit 1
EVOXMI_ANT_TRACE=1 timeout -k 10 150 python -u tools/neuro_slots.py /tmp/pop6.pt > gpurun_out/r3ab_slots.log 2>&1 || exit 1
cat gpurun_out/r3ab_slots.log | cut -c1-300
timeout -k 10 200 python -u tools/bench_neuro.py --pop 1024 --gens 10 --per-gen > gpurun_out/r3ab_pop1024_pergen.log 2>&1 || exit 1
tail -4 gpurun_out/r3ab_pop1024_pergen.log
timeout -k 10 200 python -u tools/bench_neuro.py --pop 1024 --gens 10 --graph > gpurun_out/r3ab_pop1024.log 2>&1 || exit 1
tail -1 gpurun_out/r3ab_pop1024.log
timeout -k 10 300 python -u tools/bench_neuro.py --pop 8192 --gens 10 --graph > gpurun_out/r3ab_pop8192.log 2>&1 || exit 1
tail -1 gpurun_out/r3ab_pop8192.log
timeout -k 10 200 python -u tools/neuro_latency.py 64 1024 8192 > gpurun_out/r3ab_latency.log 2>&1 || exit 1
cat gpurun_out/r3ab_latency.log
