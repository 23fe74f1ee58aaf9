set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/nds
rm -f gpurun_out/nds/probe.log
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_graph_capture_gpu.py -k "nds or moea or NSGA or nsga_select" -q --timeout 120 --timeout-method thread > gpurun_out/nds/tests.log 2>&1 || exit $?
for b in 256 64; do
  EVOXMI_NDS_BLOCKS=$b timeout -k 10 120 python tools/nds_probe.py >> gpurun_out/nds/probe.log 2>&1 || exit $?
done
timeout -k 10 300 python tools/bench_mo.py --algo nsga2 --gens 50 > gpurun_out/nds/nsga2.log 2>&1
