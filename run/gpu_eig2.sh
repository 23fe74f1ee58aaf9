set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/eig
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "jacobi or cmaes or fused_epilogue" -q --timeout 120 --timeout-method thread > gpurun_out/eig/tests.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/eig/bench.log 2>&1 || exit $?
cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES -d $GRAFT_REPO_ROOT/gpurun_out/eig/pmc -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/prof_eigh.py > $GRAFT_REPO_ROOT/gpurun_out/eig/pmc.log 2>&1
rc=$?
cd $GRAFT_REPO_ROOT
f=$(find gpurun_out/eig/pmc -name '*counter_collection.csv' | head -1)
[ -n "$f" ] && python tools/pmc_summary.py $f jacobi > gpurun_out/eig/pmc_summary.txt
find gpurun_out -name '*counter_collection.csv' -size +20M -delete
exit $rc
