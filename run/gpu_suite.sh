#!/bin/bash
# full GPU test suite (one process), then the flagship bench
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -v --timeout 200 --timeout-method thread tests -m gpu > gpurun_out/gpu_suite.log 2>&1
rc=$?; echo "suite rc=$rc"; grep -E "passed|failed" gpurun_out/gpu_suite.log | tail -3; grep -E "FAILED|ERROR" gpurun_out/gpu_suite.log | head -20
exit $rc
