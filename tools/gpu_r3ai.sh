mkdir -p gpurun_out
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "monitor" > gpurun_out/r3ai_tests.log 2>&1 || { tail -30 gpurun_out/r3ai_tests.log; exit 1; }
tail -1 gpurun_out/r3ai_tests.log
timeout -k 10 300 python -u bench.py --monitor host --phase-steps 0 > gpurun_out/r3ai_bench_mon_host.log 2>&1 || exit 1
tail -1 gpurun_out/r3ai_bench_mon_host.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('host/compute-stream', d['ms_per_step'], d['monitor'])"
EVOXMI_D2H_SIDE_STREAM=1 timeout -k 10 300 python -u bench.py --monitor host --phase-steps 0 > gpurun_out/r3ai_bench_mon_host_side.log 2>&1 || exit 1
tail -1 gpurun_out/r3ai_bench_mon_host_side.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('host/side-stream', d['ms_per_step'], d['monitor'])"
