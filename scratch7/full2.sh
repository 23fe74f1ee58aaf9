set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/s14
timeout -k 10 900 python -u -m pytest -q --timeout 400 --timeout-method thread -m gpu tests/ -x -p no:cacheprovider > gpurun_out/s14/full.log 2>&1
rc=$?
tail -30 gpurun_out/s14/full.log | cut -c1-300
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > gpurun_out/s14/b20.log 2>&1 && tail -1 gpurun_out/s14/b20.log
timeout -k 10 200 python -u bench.py --steps 50 --warmup 5 > gpurun_out/s14/b50.log 2>&1 && tail -1 gpurun_out/s14/b50.log
