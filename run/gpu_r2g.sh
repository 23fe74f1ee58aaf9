#!/bin/bash
# resume the GPU suite from the async-history test onwards, then smoke + bench + profile
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r2g
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r2g/gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r2g/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2g/smoke.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r2g/bench.log 2>&1 || exit $?
tail -1 gpurun_out/r2g/bench.log | cut -c1-250
timeout -k 10 300 python bench.py --force-dist --steps 20 --warmup 5 > gpurun_out/r2g/bench_fd.log 2>&1 || exit $?
tail -1 gpurun_out/r2g/bench_fd.log | cut -c1-250
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r2g/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 40 --warmup 5 > $GRAFT_REPO_ROOT/gpurun_out/r2g/prof_bench.log 2>&1
