set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/all
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/all/gpu_tests.log 2>&1
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/all/smoke.log 2>&1 || exit $?
timeout -k 10 300 python bench.py > gpurun_out/all/bench.log 2>&1 || exit $?
timeout -k 10 300 python tools/bench_neuro.py --gens 5 --graph > gpurun_out/all/neuro.log 2>&1 || exit $?
timeout -k 10 300 python tools/bench_mo.py --algo nsga2 --gens 50 > gpurun_out/all/nsga2.log 2>&1 || exit $?
timeout -k 10 300 python tools/bench_mo.py --algo moead --gens 20 > gpurun_out/all/moead.log 2>&1 || exit $?
