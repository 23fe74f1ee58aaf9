#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r2f
timeout -k 10 500 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_eigh_sbr.py tests/test_kernels_gpu.py -m gpu -k "sbr or taylor or jacobi or cmaes or ant or openes" > gpurun_out/r2f/tests.log 2>&1
rc=$?; tail -3 gpurun_out/r2f/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/bench_neuro.py --gens 5 --graph > gpurun_out/r2f/neuro.log 2>&1 || exit $?
tail -1 gpurun_out/r2f/neuro.log | cut -c1-300
timeout -k 10 240 python bench.py --steps 20 --warmup 5 > gpurun_out/r2f/bench20.log 2>&1 || exit $?
tail -1 gpurun_out/r2f/bench20.log | cut -c1-250
timeout -k 10 240 python bench.py > gpurun_out/r2f/bench50.log 2>&1 || exit $?
tail -1 gpurun_out/r2f/bench50.log | cut -c1-250; tail -1 gpurun_out/r2f/bench50.log | grep -o '"phases.*'
