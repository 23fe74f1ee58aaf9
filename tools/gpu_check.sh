#!/bin/bash
# One GPU-box session: build, GPU tests, short bench, rocprof kernel stats.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -m evoxmi.ops.build > gpurun_out/build.log 2>&1 || { echo BUILD FAILED; tail -30 gpurun_out/build.log; exit 1; }
echo "== pytest -m gpu"
timeout -k 10 600 python -m pytest tests -x -q -m gpu ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -25 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && [ $rc -ne 5 ] && exit $rc
echo "== smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -30 gpurun_out/smoke.log; exit 1; }
tail -2 gpurun_out/smoke.log
echo "== bench"
timeout -k 10 300 python bench.py --steps ${STEPS:-20} --warmup ${WARMUP:-3} ${BENCH_ARGS} > gpurun_out/bench.log 2>&1 || { tail -30 gpurun_out/bench.log; exit 1; }
cat gpurun_out/bench.log | tail -3
if [ -n "$PROFILE" ]; then
  echo "== rocprof"
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 2 ${BENCH_ARGS} > $GRAFT_REPO_ROOT/gpurun_out/prof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/prof.log; exit 1; }
  cd $GRAFT_REPO_ROOT
  f=$(find gpurun_out/prof -name '*kernel_stats.csv' | head -1); [ -n "$f" ] && head -25 "$f"
fi
