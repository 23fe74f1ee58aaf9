set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/round
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/round/gpu_tests.log 2>&1
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/round/smoke.log 2>&1 || exit $?
timeout -k 10 300 python bench.py > gpurun_out/round/bench.log 2>&1
