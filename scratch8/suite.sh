set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/suite
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/suite/smoke.log 2>&1 || { tail -20 gpurun_out/suite/smoke.log; exit 1; }
tail -1 gpurun_out/suite/smoke.log
timeout -k 10 1500 python -u -m pytest -q --timeout 400 --timeout-method thread -m gpu tests/ -p no:cacheprovider > gpurun_out/suite/full.log 2>&1
rc=$?
tail -8 gpurun_out/suite/full.log | cut -c1-300
exit $rc
