mkdir -p gpurun_out
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_workflows.py tests/test_neuroevolution.py -m gpu -x -q --timeout 120 --timeout-method thread -k "monitor or Monitor" > gpurun_out/r3ah_tests.log 2>&1 || { tail -30 gpurun_out/r3ah_tests.log; exit 1; }
tail -1 gpurun_out/r3ah_tests.log
for m in host device; do
timeout -k 10 300 python -u bench.py --monitor $m --phase-steps 0 > gpurun_out/r3ah_bench_mon_$m.log 2>&1 || exit 1
tail -1 gpurun_out/r3ah_bench_mon_$m.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$m', d['ms_per_step'], d['monitor'])"
done
