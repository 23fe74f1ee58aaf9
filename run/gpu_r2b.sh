#!/bin/bash
# round-2 re-entry check: GPU suite, smoke, bench and a kernel-stats profile of bench.py
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r2b
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2b/gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r2b/gpu_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2b/smoke.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/r2b/bench.log 2>&1 || exit $?
tail -1 gpurun_out/r2b/bench.log
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r2b/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 3 > $GRAFT_REPO_ROOT/gpurun_out/r2b/prof_bench.log 2>&1
