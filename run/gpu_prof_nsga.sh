set -o pipefail
cd $GRAFT_REPO_ROOT
TOPN=25 bash tools/prof.sh nsga2 $GRAFT_REPO_ROOT/tools/bench_mo.py --algo nsga2 --gens 50 --no-graph
rc=$?
find gpurun_out -name '*kernel_trace.csv' -delete
exit $rc
