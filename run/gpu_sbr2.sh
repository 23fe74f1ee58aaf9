#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/bench_sbr.py > gpurun_out/bench_sbr_parts.log 2>&1
rc=$?; echo "bench_sbr rc=$rc"; cat gpurun_out/bench_sbr_parts.log | cut -c1-400
[ $rc -ne 0 ] && exit $rc
timeout -k 10 420 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_eigh_sbr.py -m gpu > gpurun_out/sbr_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -15 gpurun_out/sbr_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 240 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_sbr.log 2>&1
rc2=$?; echo "bench rc=$rc2"; tail -1 gpurun_out/bench_sbr.log
exit $rc2
