# CMA-ES graph path: population / invsqrtC written in place (no write-back copy) — tests + bench + copy count
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "cma or CMA or graph or determinism or eigh or bench or workflow" > gpurun_out/r3au_tests.log 2>&1 || { tail -40 gpurun_out/r3au_tests.log; exit 1; }
tail -2 gpurun_out/r3au_tests.log
for i in 1 2; do
timeout -k 10 300 python bench.py --steps 50 --warmup 3 > gpurun_out/r3au_bench50_$i.log 2>&1 || { tail -30 gpurun_out/r3au_bench50_$i.log; exit 1; }
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('50 steps', d['ms_per_step'], d['eigh_stats']['max_off_rel'])" gpurun_out/r3au_bench50_$i.log
done
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/r3au_bench20.log 2>&1 || { tail -30 gpurun_out/r3au_bench20.log; exit 1; }
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('20 steps', d['ms_per_step'])" gpurun_out/r3au_bench20.log
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r3au_prof -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 3 > $R/gpurun_out/r3au_prof.log 2>&1 || { tail -20 $R/gpurun_out/r3au_prof.log; exit 1; }
cd $R && python tools/kstats.py $(find gpurun_out/r3au_prof -name '*kernel_stats.csv' | head -1) 23 40 > gpurun_out/r3au_kstats.txt 2>&1; grep -iE "copy|multi_tensor|total" gpurun_out/r3au_kstats.txt
