#!/bin/bash
# Batched independent DE runs on one MI355X: identity tests, then aggregate throughput
# of run/run_de.py --batched (32 runs, D=20, pop=100) vs the sequential harness.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_batched_runs.py -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/batched_tests.log 2>&1 || { tail -40 gpurun_out/batched_tests.log; exit 1; }
tail -3 gpurun_out/batched_tests.log
for A in EVDE LSHADE; do
  timeout -k 10 300 python -u run/run_de.py --algo $A --funcs 1-1 --dim 20 --pop 100 --runs 32 --batched \
    --max-steps 2000 --progress steps --max-time 1e9 --sync-every 100 --out gpurun_out/rde_b_$A --json gpurun_out/rde_b_$A.json \
    > gpurun_out/rde_b_$A.log 2>&1 || { tail -30 gpurun_out/rde_b_$A.log; exit 1; }
  tail -2 gpurun_out/rde_b_$A.log
  timeout -k 10 300 python -u run/run_de.py --algo $A --funcs 1-1 --dim 20 --pop 100 --runs 8 \
    --max-steps 500 --progress steps --max-time 1e9 --sync-every 100 --out gpurun_out/rde_s_$A --json gpurun_out/rde_s_$A.json \
    > gpurun_out/rde_s_$A.log 2>&1 || { tail -30 gpurun_out/rde_s_$A.log; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/rde_s_$A.json')); print('$A sequential', {k: v['gens_per_s_aggregate'] for k, v in d['functions'].items()})"
done
