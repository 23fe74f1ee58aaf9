set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/inner
EVOXMI_JACOBI_INNER=2 timeout -k 10 300 python tools/eig_probe.py 21 > gpurun_out/inner/probe_inner2.log 2>&1 || exit $?
EVOXMI_JACOBI_INNER=3 timeout -k 10 300 python tools/eig_probe.py 21 > gpurun_out/inner/probe_inner3.log 2>&1 || exit $?
