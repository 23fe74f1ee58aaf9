set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/de
for k in 1 4 8 16; do
  timeout -k 10 200 python run/run_de.py --algo SHADE --funcs 1 --runs $k --max-time 4 --concurrent $k --out /tmp/rde_$k > gpurun_out/de/conc_$k.log 2>&1 || exit $?
done
for k in 1 8; do
  timeout -k 10 200 python run/run_de.py --algo LSHADE --funcs 1 --runs $k --max-time 4 --concurrent $k --out /tmp/rdl_$k > gpurun_out/de/lconc_$k.log 2>&1 || exit $?
done
