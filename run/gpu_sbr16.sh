#!/bin/bash
# 16-block SBR: kernel tests, part timings, converged solve timings and the flagship bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/sbr16
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_eigh_sbr.py -m gpu -k "sbr16 or stats or converges" > gpurun_out/sbr16/tests.log 2>&1
rc=$?; tail -8 gpurun_out/sbr16/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 240 python -u tools/bench_sbr.py > gpurun_out/sbr16/parts.log 2>&1 || exit $?
cut -c1-400 gpurun_out/sbr16/parts.log
timeout -k 10 240 python bench.py --steps 30 --warmup 5 > gpurun_out/sbr16/bench.log 2>&1 || exit $?
tail -1 gpurun_out/sbr16/bench.log
