#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/neuro2
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "ant or openes" > gpurun_out/neuro2/tests.log 2>&1
rc=$?; tail -2 gpurun_out/neuro2/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/bench_neuro.py --gens 5 --graph > gpurun_out/neuro2/neuro.log 2>&1 || exit $?
tail -1 gpurun_out/neuro2/neuro.log | cut -c1-300
timeout -k 10 300 python tools/bench_neuro.py --gens 3 --graph --kernel-only > gpurun_out/neuro2/neuro_kernel.log 2>&1; tail -1 gpurun_out/neuro2/neuro_kernel.log | cut -c1-300
