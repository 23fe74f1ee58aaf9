#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/f2
timeout -k 10 500 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_eigh_sbr.py tests/test_determinism_gpu.py tests/test_kernels_gpu.py -m gpu -k "sbr or determin or jacobi or cmaes or eigh" > gpurun_out/f2/tests.log 2>&1
rc=$?; tail -2 gpurun_out/f2/tests.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --phase-steps 0 > gpurun_out/f2/bench.$i.log 2>&1 || exit $?
tail -1 gpurun_out/f2/bench.$i.log | grep -o '"ms_per_step": [0-9.]*\|"max_off_rel": [0-9.e-]*'
done
