mkdir -p gpurun_out
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_moead_sharded.py -q --timeout 250 --timeout-method thread -m gpu > gpurun_out/r3e_tests.log 2>&1; tail -2 gpurun_out/r3e_tests.log

timeout -k 10 200 python -u tools/bench_mo.py --algo moead --gens 10 --warmup 2 --simulate-rank 0 --world 8 --shard owner > gpurun_out/moead_sim8_owner.log 2>&1 || exit 1; tail -1 gpurun_out/moead_sim8_owner.log
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_moead_sim8 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/bench_mo.py --algo moead --gens 10 --warmup 2 --simulate-rank 0 --world 8 --shard owner > $GRAFT_REPO_ROOT/gpurun_out/prof_moead_sim8.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT && f=$(find gpurun_out/prof_moead_sim8 -name '*kernel_stats.csv' | head -1) && python tools/kstats.py $f 13 18
