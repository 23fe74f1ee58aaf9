#!/bin/bash
# planned SBR solves: tests, variant trajectory on bench matrices, bench with 16- and 64-blocks
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/sbr16b
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_eigh_sbr.py -m gpu -k "sbr16 or stats or converges or damping" > gpurun_out/sbr16b/tests.log 2>&1
rc=$?; tail -3 gpurun_out/sbr16b/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u tools/sbr_traj.py --gens 35 --variants 16:0.3:0:3,16:0.3:0:0,64:0.3:0:3 > gpurun_out/sbr16b/traj.log 2>&1 || exit $?
tail -1 gpurun_out/sbr16b/traj.log
timeout -k 10 240 python bench.py --steps 30 --warmup 5 > gpurun_out/sbr16b/bench16.log 2>&1 || exit $?
tail -1 gpurun_out/sbr16b/bench16.log | cut -c 1-200; tail -1 gpurun_out/sbr16b/bench16.log | grep -o '"phases.*'
EVOXMI_SBR_BLOCK=64 timeout -k 10 240 python bench.py --steps 30 --warmup 5 > gpurun_out/sbr16b/bench64.log 2>&1 || exit $?
tail -1 gpurun_out/sbr16b/bench64.log | cut -c 1-200; tail -1 gpurun_out/sbr16b/bench64.log | grep -o '"phases.*'
