#!/bin/bash
# articulated Ant kernel vs oracle, SBR kernels, neuro bench, flagship bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r2c
timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_eigh_sbr.py -m gpu -k "ant or openes or sbr16 or damping or converges" > gpurun_out/r2c/tests.log 2>&1
rc=$?; grep -E "passed|failed|FAILED|Error" gpurun_out/r2c/tests.log | tail -12
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python tools/bench_neuro.py --gens 5 --graph > gpurun_out/r2c/neuro.log 2>&1 || exit $?
tail -1 gpurun_out/r2c/neuro.log | cut -c1-400
timeout -k 10 240 python bench.py --steps 30 --warmup 5 > gpurun_out/r2c/bench.log 2>&1 || exit $?
tail -1 gpurun_out/r2c/bench.log | cut -c1-200; tail -1 gpurun_out/r2c/bench.log | grep -o '"phases.*'
