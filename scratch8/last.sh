set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/last
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/last/smoke.log 2>&1 || { tail -20 gpurun_out/last/smoke.log; exit 1; }
tail -1 gpurun_out/last/smoke.log
timeout -k 10 200 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/last/b20.log 2>&1 || { tail -5 gpurun_out/last/b20.log; exit 1; }
tail -1 gpurun_out/last/b20.log | cut -c1-400
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread -x -p no:cacheprovider tests/test_gemm_blk.py tests/test_kernels_gpu.py -k "h3 or blk or cec2022" > gpurun_out/last/t.log 2>&1; rc=$?; tail -1 gpurun_out/last/t.log; exit $rc
