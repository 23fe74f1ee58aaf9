#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r2d
timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_eigh_sbr.py -m gpu > gpurun_out/r2d/tests.log 2>&1
rc=$?; grep -E "passed|failed|FAILED|Error" gpurun_out/r2d/tests.log | tail -6
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 240 python bench.py --steps 30 --warmup 5 > gpurun_out/r2d/bench.log 2>&1 || exit $?
tail -1 gpurun_out/r2d/bench.log | cut -c1-200; tail -1 gpurun_out/r2d/bench.log | grep -o '"phases.*'
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r2d/p -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 40 --warmup 5 > $GRAFT_REPO_ROOT/gpurun_out/r2d/prof_bench.log 2>&1
