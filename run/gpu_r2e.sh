#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r2e
timeout -k 10 400 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_eigh_sbr.py -m gpu > gpurun_out/r2e/tests.log 2>&1
rc=$?; tail -2 gpurun_out/r2e/tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 240 python bench.py --steps 20 --warmup 5 > gpurun_out/r2e/bench20.log 2>&1 || exit $?
tail -1 gpurun_out/r2e/bench20.log | cut -c1-250
timeout -k 10 240 python bench.py > gpurun_out/r2e/bench50.log 2>&1 || exit $?
tail -1 gpurun_out/r2e/bench50.log | cut -c1-250; tail -1 gpurun_out/r2e/bench50.log | grep -o '"phases.*'
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r2e/p -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 40 --warmup 5 > $GRAFT_REPO_ROOT/gpurun_out/r2e/prof_bench.log 2>&1
