#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/wrs
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "weighted_rowsum or cmaes" > gpurun_out/wrs/tests.log 2>&1
rc=$?; tail -1 gpurun_out/wrs/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/wrs/bench.log 2>&1 || exit $?
tail -1 gpurun_out/wrs/bench.log | cut -c1-230
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/wrs/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 3 > $GRAFT_REPO_ROOT/gpurun_out/wrs/prof_bench.log 2>&1
