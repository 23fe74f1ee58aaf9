set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/eig
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "jacobi or cmaes or argsort or gemm or cec" -v --timeout 120 --timeout-method thread > gpurun_out/eig/tests.log 2>&1
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python tools/eig_probe.py 31 > gpurun_out/eig/probe.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/eig/bench.log 2>&1 || exit $?
TOPN=14 bash tools/prof.sh cma $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 3
rc=$?
find gpurun_out -name '*kernel_trace.csv' -delete
exit $rc
