set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/mo
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "moead or lsmop or nds or sbx or pm or moea" -v --timeout 60 --timeout-method thread > gpurun_out/mo/k_tests.log 2>&1
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python -u -m pytest tests/test_graph_capture_gpu.py -q --timeout 120 --timeout-method thread > gpurun_out/mo/graph_tests.log 2>&1
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python tools/bench_mo.py --algo moead --gens 10 > gpurun_out/mo/moead.log 2>&1 || exit $?
TOPN=30 bash tools/prof.sh moead $GRAFT_REPO_ROOT/tools/bench_mo.py --algo moead --gens 5 --no-graph
rc=$?
find gpurun_out -name '*kernel_trace.csv' -delete
exit $rc
