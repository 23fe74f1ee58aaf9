#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 250 --timeout-method thread tests/test_moead_sharded.py -m gpu > gpurun_out/moead_sharded_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/moead_sharded_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python tools/bench_mo.py --algo moead --gens 10 --warmup 2 > gpurun_out/moead_single.log 2>&1; rc=$?; tail -1 gpurun_out/moead_single.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29551 tools/bench_mo.py --algo moead --gens 10 --warmup 2 --force-dist > gpurun_out/moead_forcedist.log 2>&1; rc=$?; grep "^{" gpurun_out/moead_forcedist.log; tail -2 gpurun_out/moead_forcedist.log
exit $rc
