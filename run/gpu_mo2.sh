#!/bin/bash
# multi-objective north-star configs after the round-2 changes (NSGA-II DTLZ2, MOEA/D LSMOP1)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/mo2
timeout -k 10 300 python tools/bench_mo.py --algo nsga2 --gens 50 > gpurun_out/mo2/nsga2.log 2>&1 || exit $?
tail -1 gpurun_out/mo2/nsga2.log | cut -c1-300
timeout -k 10 300 python tools/bench_mo.py --algo moead --gens 30 > gpurun_out/mo2/moead.log 2>&1 || exit $?
tail -1 gpurun_out/mo2/moead.log | cut -c1-300
