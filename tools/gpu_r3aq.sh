# fused damping + column PSO + distributed bench checks
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_sbr_device_gpu.py tests/test_determinism_gpu.py tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "sbr or determinism or bit_identical or pso or cmaes or de_trial" > gpurun_out/r3aq_tests.log 2>&1 || { tail -30 gpurun_out/r3aq_tests.log; exit 1; }
tail -1 gpurun_out/r3aq_tests.log
timeout -k 10 300 python -u bench.py > gpurun_out/r3aq_bench.log 2>&1 || exit 1
tail -1 gpurun_out/r3aq_bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench', d['ms_per_step'], d['eigh_stats'])"
EVOXMI_SBR_FUSED_DAMPING=0 timeout -k 10 300 python -u bench.py > gpurun_out/r3aq_bench_unfused.log 2>&1 || exit 1
tail -1 gpurun_out/r3aq_bench_unfused.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench 4-launch damping', d['ms_per_step'], d['eigh_stats'])"
timeout -k 10 300 python -u bench.py --force-dist > gpurun_out/r3aq_forcedist.log 2>&1 || exit 1
tail -1 gpurun_out/r3aq_forcedist.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('force-dist', d['ms_per_step'], d['config']['parallelism'])"
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --steps 20 --warmup 3 > gpurun_out/r3aq_torchrun1.log 2>&1 || exit 1
tail -1 gpurun_out/r3aq_torchrun1.log | cut -c1-250
