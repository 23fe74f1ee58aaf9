set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/s13
timeout -k 10 1140 python -u -m pytest -q --timeout 400 --timeout-method thread -m gpu tests/ -x -p no:cacheprovider > gpurun_out/s13/full.log 2>&1
rc=$?
tail -30 gpurun_out/s13/full.log | cut -c1-300
exit $rc
