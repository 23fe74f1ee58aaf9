set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/sp
for inner in 0 1; do
  EVOXMI_JACOBI_INNER=$inner timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/sp/i$inner -o run --output-format csv -- python3 tools/prof_eigh.py > gpurun_out/sp/i$inner.log 2>&1 || exit $?
done
python3 tools/kstats.py $(find gpurun_out/sp/i0 -name "*kernel_stats.csv") 3 8 > gpurun_out/sp/k0.txt 2>&1; python3 tools/kstats.py $(find gpurun_out/sp/i1 -name "*kernel_stats.csv") 3 8 > gpurun_out/sp/k1.txt 2>&1; true
