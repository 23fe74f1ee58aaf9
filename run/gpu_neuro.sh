set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/neuro
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "openes or ant" -v --timeout 120 --timeout-method thread > gpurun_out/neuro/tests.log 2>&1
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python tools/bench_neuro.py --gens 5 > gpurun_out/neuro/eager.log 2>&1 || exit $?
timeout -k 10 300 python tools/bench_neuro.py --gens 5 --graph > gpurun_out/neuro/graph.log 2>&1 || exit $?
TOPN=15 bash tools/prof.sh neuro $GRAFT_REPO_ROOT/tools/bench_neuro.py --gens 3
rc=$?
find gpurun_out -name '*kernel_trace.csv' -delete
exit $rc
