set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/trace
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/trace/cma -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-graph > $GRAFT_REPO_ROOT/gpurun_out/trace/cma.log 2>&1
rc=$?
cd $GRAFT_REPO_ROOT
f=$(find gpurun_out/trace/cma -name '*kernel_trace.csv' | head -1)
[ -n "$f" ] && python tools/ktrace_tail.py $f > gpurun_out/trace/cma_lastgen.txt
find gpurun_out -name '*kernel_trace.csv' -delete
exit $rc
