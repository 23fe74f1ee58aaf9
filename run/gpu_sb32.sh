#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/sb32
timeout -k 10 400 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_eigh_sbr.py -m gpu > gpurun_out/sb32/tests.log 2>&1
rc=$?; tail -2 gpurun_out/sb32/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u tools/sbr_traj.py --gens 35 --variants 16:0.3:0:3,32:0.3:0:3 > gpurun_out/sb32/traj.log 2>&1 || exit $?
tail -1 gpurun_out/sb32/traj.log
for i in 1 2; do
  for b in 16 32; do
    EVOXMI_SBR_BLOCK=$b timeout -k 10 300 python bench.py --steps 20 --warmup 5 --phase-steps 0 > gpurun_out/sb32/b$b.20.$i.log 2>&1 || exit $?
    EVOXMI_SBR_BLOCK=$b timeout -k 10 300 python bench.py --steps 50 --warmup 5 --phase-steps 0 > gpurun_out/sb32/b$b.50.$i.log 2>&1 || exit $?
    echo "block $b run $i: 20 steps $(tail -1 gpurun_out/sb32/b$b.20.$i.log | grep -o '"ms_per_step": [0-9.]*') 50 steps $(tail -1 gpurun_out/sb32/b$b.50.$i.log | grep -o '"ms_per_step": [0-9.]*') iters $(tail -1 gpurun_out/sb32/b$b.50.$i.log | grep -o '"mean_refine_iters": [0-9.]*')"
  done
done
