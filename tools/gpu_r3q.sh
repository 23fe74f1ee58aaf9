# PMC pass over OpenES pop 1024 generations: is the slow regime clock or stalls?
mkdir -p gpurun_out/pmc
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
C="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT"
cd /tmp && timeout -s KILL 200 rocprofv3 --kernel-trace --pmc $C -d $R/gpurun_out/pmc/antgen_p1 -o run --output-format csv -- python3 $R/tools/bench_neuro.py --pop 1024 --gens 5 --per-gen > $R/gpurun_out/pmc/antgen_p1.log 2>&1
rc=$?; cd $R; tail -7 gpurun_out/pmc/antgen_p1.log; exit $rc
