#!/bin/bash
# PyTorch TunableOp: tune every hipBLASLt/rocBLAS GEMM shape of the flagship once, then
# bench with the tuned table (tuning off) against the default heuristics on the same box
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/tune
export PYTORCH_TUNABLEOP_FILENAME=$GRAFT_REPO_ROOT/gpurun_out/tune/tunableop_results%d.csv
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/tune/bench_default.log 2>&1 || exit $?
tail -1 gpurun_out/tune/bench_default.log | cut -c1-220
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=30 timeout -k 10 600 python bench.py --no-graph --steps 3 --warmup 2 --phase-steps 0 > gpurun_out/tune/tuning.log 2>&1 || exit $?
ls -la gpurun_out/tune/; wc -l gpurun_out/tune/*.csv
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=0 timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/tune/bench_tuned.log 2>&1 || exit $?
tail -1 gpurun_out/tune/bench_tuned.log | cut -c1-220
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=0 timeout -k 10 300 python bench.py --steps 50 --warmup 5 > gpurun_out/tune/bench_tuned50.log 2>&1 || exit $?
tail -1 gpurun_out/tune/bench_tuned50.log | cut -c1-220
