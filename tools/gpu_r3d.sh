set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_sbr_device_gpu.py tests/test_moead_sharded.py tests/test_kernels_gpu.py -q --timeout 250 --timeout-method thread -m gpu -k "cmaes or sbr or device or moead" > gpurun_out/r3d_tests.log 2>&1; tail -3 gpurun_out/r3d_tests.log
for w in 2 4 8; do timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --simulate-rank 0 --world $w > gpurun_out/sim_rank0_world$w.log 2>&1 || exit 1; tail -1 gpurun_out/sim_rank0_world$w.log | cut -c 1-1500; done
timeout -k 10 200 python -u tools/bench_mo.py --algo moead --gens 10 --warmup 2 > gpurun_out/moead_single.log 2>&1 || exit 1; tail -1 gpurun_out/moead_single.log
timeout -k 10 200 python -u tools/bench_mo.py --algo moead --gens 10 --warmup 2 --simulate-rank 0 --world 8 --shard owner > gpurun_out/moead_sim8_owner.log 2>&1 || exit 1; tail -1 gpurun_out/moead_sim8_owner.log
timeout -k 10 200 python -u tools/bench_mo.py --algo moead --gens 10 --warmup 2 --simulate-rank 0 --world 8 --shard replica > gpurun_out/moead_sim8_replica.log 2>&1 || exit 1; tail -1 gpurun_out/moead_sim8_replica.log
