#!/bin/bash
# SBR eigensolver: GPU tests + flagship bench (each step time-limited; stop on a crash/timeout)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_eigh_sbr.py -m gpu > gpurun_out/sbr_tests.log 2>&1
rc=$?
echo "tests rc=$rc"
tail -5 gpurun_out/sbr_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 240 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_sbr.log 2>&1
rc2=$?
echo "bench rc=$rc2"
tail -3 gpurun_out/bench_sbr.log
[ $rc2 -ne 0 ] && exit $rc2
TOPN=30 bash tools/prof.sh sbr_bench "$PWD/bench.py" --steps 10 --warmup 3

