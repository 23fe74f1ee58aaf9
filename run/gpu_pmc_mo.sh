set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
R=$GRAFT_REPO_ROOT
cd /tmp && timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE -d $R/gpurun_out/pmc/fetch -o run --output-format csv -- python3 $R/tools/bench_mo.py --algo moead --gens 3 --warmup 1 --no-graph > $R/gpurun_out/pmc/fetch.log 2>&1 || exit $?
cd /tmp && timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE SQ_WAVE_CYCLES SQ_INSTS_VALU -d $R/gpurun_out/pmc/write -o run --output-format csv -- python3 $R/tools/bench_mo.py --algo moead --gens 3 --warmup 1 --no-graph > $R/gpurun_out/pmc/write.log 2>&1 || exit $?
cd $R
for p in fetch write; do
  f=$(find gpurun_out/pmc/$p -name '*counter_collection.csv' | head -1)
  [ -n "$f" ] && python tools/pmc_summary.py $f > gpurun_out/pmc/${p}_summary.txt
done
find gpurun_out/pmc -name '*counter_collection.csv' -delete
