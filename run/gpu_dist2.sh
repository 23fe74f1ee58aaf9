set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/dist
timeout -k 10 600 python -u -m pytest tests/test_distributed_gpu.py -v --timeout 300 --timeout-method thread > gpurun_out/dist/tests.log 2>&1
