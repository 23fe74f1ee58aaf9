set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/pmce
R=$GRAFT_REPO_ROOT
cd /tmp && timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES -d $R/gpurun_out/pmce/sq -o run --output-format csv -- python3 $R/tools/prof_eigh.py > $R/gpurun_out/pmce/sq.log 2>&1 || exit $?
cd /tmp && timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE -d $R/gpurun_out/pmce/fetch -o run --output-format csv -- python3 $R/tools/prof_eigh.py > $R/gpurun_out/pmce/fetch.log 2>&1 || exit $?
cd $R
for p in sq fetch; do
  f=$(find gpurun_out/pmce/$p -name '*counter_collection.csv' | head -1)
  [ -n "$f" ] && python tools/pmc_summary.py $f > gpurun_out/pmce/${p}_summary.txt
done
find gpurun_out/pmce -name '*counter_collection.csv' -delete
true
