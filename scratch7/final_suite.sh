set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/s22
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/s22/smoke.log 2>&1 || { tail -20 gpurun_out/s22/smoke.log; exit 1; }
tail -1 gpurun_out/s22/smoke.log
timeout -k 10 900 python -u -m pytest -q --timeout 400 --timeout-method thread -m gpu tests/ -x -p no:cacheprovider > gpurun_out/s22/full.log 2>&1
rc=$?
tail -5 gpurun_out/s22/full.log | cut -c1-300
exit $rc
