set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/eig
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "jacobi or cmaes" -v --timeout 120 --timeout-method thread > gpurun_out/eig/tests.log 2>&1
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python tools/eig_probe.py 61 > gpurun_out/eig/probe.log 2>&1 || exit $?
EVOXMI_JACOBI_SOLVER=256 timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/eig/bench_256.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/eig/bench_64.log 2>&1
