#!/bin/bash
# A/B: default hipBLASLt heuristics vs the committed TunableOp table, alternating runs
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/ab
for i in 1 2; do
  for mode in default tuned; do
    if [ $mode = tuned ]; then
      export PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=0 PYTORCH_TUNABLEOP_FILENAME=$GRAFT_REPO_ROOT/evoxmi/tuning/tunableop_mi355x.csv
    else
      unset PYTORCH_TUNABLEOP_ENABLED PYTORCH_TUNABLEOP_TUNING PYTORCH_TUNABLEOP_FILENAME
    fi
    for steps in 20 50; do
      timeout -k 10 300 python bench.py --steps $steps --warmup 5 --phase-steps 0 > gpurun_out/ab/$mode.$steps.$i.log 2>&1 || exit $?
      echo "$mode $steps $i $(tail -1 gpurun_out/ab/$mode.$steps.$i.log | grep -o '"ms_per_step": [0-9.]*')"
    done
  done
done
