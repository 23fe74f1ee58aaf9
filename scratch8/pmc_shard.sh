mkdir -p gpurun_out/pmc
set -o pipefail
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE GRBM_COUNT"
for W in 2 8; do
  cd /tmp && timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $P1 -d $R/gpurun_out/pmc/sim${W}_p1 -o run --output-format csv -- python3 $R/bench.py --simulate-rank 0 --world $W --steps 3 --warmup 1 --no-graph --phase-steps 0 > $R/gpurun_out/pmc/sim${W}_p1.log 2>&1
  rc=$?; cd $R; echo "sim$W rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/pmc/sim${W}_p1.log; exit 1; }
  python tools/pmc_summary.py gpurun_out/pmc/sim${W}_summary.txt gpurun_out/pmc/sim${W}_p1 > /dev/null || exit 1
  grep -i "gemm_h3\|Kernel\|kernel " gpurun_out/pmc/sim${W}_summary.txt | head -6 | cut -c1-220
done
