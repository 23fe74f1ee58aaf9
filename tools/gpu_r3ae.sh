mkdir -p gpurun_out
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_graph_capture_gpu.py tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "cec2022_generation or eval_monitor" > gpurun_out/r3ae_tests.log 2>&1 || { tail -30 gpurun_out/r3ae_tests.log; exit 1; }
tail -1 gpurun_out/r3ae_tests.log
timeout -k 10 300 python -u bench.py --monitor host --phase-steps 0 > gpurun_out/r3ae_bench_mon_host.log 2>&1 || exit 1
tail -1 gpurun_out/r3ae_bench_mon_host.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('host', d['ms_per_step'], d['monitor'])"
