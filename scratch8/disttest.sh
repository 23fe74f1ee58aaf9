set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/disttest
timeout -k 10 400 python -u -m pytest -q --timeout 300 --timeout-method thread -x -p no:cacheprovider tests/test_distributed_gpu.py -k "flagship or match_single" > gpurun_out/disttest/t.log 2>&1; rc=$?
tail -3 gpurun_out/disttest/t.log | cut -c1-300; [ $rc -ne 0 ] && grep -m5 "Error\|assert" gpurun_out/disttest/t.log | cut -c1-300
exit $rc
