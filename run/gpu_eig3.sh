set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/eig3
timeout -k 10 300 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/eig3/tests.log 2>&1 || exit $?
timeout -k 10 300 python bench.py > gpurun_out/eig3/bench.log 2>&1 || exit $?
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/eig3/prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 > gpurun_out/eig3/prof.log 2>&1 || exit $?
python3 tools/kstats.py $(find gpurun_out/eig3/prof -name "*kernel_stats.csv") 23 12 > gpurun_out/eig3/k.txt 2>&1; true
