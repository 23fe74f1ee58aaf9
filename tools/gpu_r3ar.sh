# MOEA/D graph path: in-place offspring / winner rows (no state write-back copies)
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_graph_capture_gpu.py tests/test_moead_sharded.py tests/test_determinism_gpu.py tests/test_kernels_gpu.py tests/test_lsmop.py -m gpu -x -q --timeout 200 --timeout-method thread -k "MOEAD or moead or determinism or bit_identical or lsmop or LSMOP" > gpurun_out/r3ar_tests.log 2>&1 || { tail -30 gpurun_out/r3ar_tests.log; exit 1; }
tail -1 gpurun_out/r3ar_tests.log
timeout -k 10 300 python -u tools/bench_mo.py --algo moead --gens 20 --warmup 3 > gpurun_out/r3ar_moead_single.log 2>&1 || exit 1
tail -1 gpurun_out/r3ar_moead_single.log | cut -c1-300
timeout -k 10 300 python -u tools/bench_mo.py --algo moead --gens 10 --warmup 2 --simulate-rank 0 --world 8 --shard owner > gpurun_out/r3ar_moead_sim8.log 2>&1 || exit 1
tail -1 gpurun_out/r3ar_moead_sim8.log | cut -c1-250
timeout -k 10 300 python -u tools/bench_mo.py --algo nsga2 --gens 20 --warmup 3 > gpurun_out/r3ar_nsga2.log 2>&1 || exit 1
tail -1 gpurun_out/r3ar_nsga2.log | cut -c1-250
