set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TOPN=30 bash tools/prof.sh nsga2 $GRAFT_REPO_ROOT/tools/bench_mo.py --algo nsga2 --gens 10 --no-graph && \
TOPN=30 bash tools/prof.sh moead $GRAFT_REPO_ROOT/tools/bench_mo.py --algo moead --gens 5 --no-graph
rc=$?
find gpurun_out -name '*kernel_trace.csv' -delete
exit $rc
