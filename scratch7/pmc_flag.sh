# rocprofv3 PMC passes (kernel trace + counters only; no sys/runtime traces) over the
# flagship (eager, so every dispatch is its own record), MOEA/D owner-mode rank share and
# the Ant rollout.  One pass per counter group, each under its own SIGKILL limit.
mkdir -p gpurun_out/pmc6
set -o pipefail
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE GRBM_COUNT"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_SMEM FETCH_SIZE"
P3="WRITE_SIZE TCC_HIT_sum TCC_MISS_sum"
run() {  # name, pass index, counters, program...
  local name=$1 p=$2 c=$3; shift 3
  cd /tmp && timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $c -d $R/gpurun_out/pmc6/${name}_p$p -o run --output-format csv -- "$@" > $R/gpurun_out/pmc6/${name}_p$p.log 2>&1
  local rc=$?; cd $R; echo "$name pass $p rc=$rc"; return $rc
}
for p in 1 2 3; do
  eval c=\$P$p
  run flagship $p "$c" python3 $R/bench.py --steps 3 --warmup 1 --no-graph --phase-steps 0 || exit 1
done
python tools/pmc_summary.py gpurun_out/pmc6/flagship_summary.txt gpurun_out/pmc6/flagship_p1 gpurun_out/pmc6/flagship_p2 gpurun_out/pmc6/flagship_p3 > /dev/null || exit 1
head -45 gpurun_out/pmc6/flagship_summary.txt | cut -c1-200
