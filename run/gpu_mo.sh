set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/mo
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_graph_capture_gpu.py -k "nds or moea or NSGA" -q --timeout 120 --timeout-method thread > gpurun_out/mo/k_tests.log 2>&1 || exit $?
timeout -k 10 300 python tools/bench_mo.py --algo nsga2 --gens 50 > gpurun_out/mo/nsga2.log 2>&1 || exit $?
TOPN=12 bash tools/prof.sh nsga2 $GRAFT_REPO_ROOT/tools/bench_mo.py --algo nsga2 --gens 20 --no-graph
rc=$?
find gpurun_out -name '*kernel_trace.csv' -delete
exit $rc
