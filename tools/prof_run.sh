set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -m evoxmi.ops.build > gpurun_out/build.log 2>&1 || { tail -30 gpurun_out/build.log; exit 1; }
timeout -k 10 300 python -m pytest tests -x -q -m gpu -k "ant" > gpurun_out/pytest_ant.log 2>&1; tail -3 gpurun_out/pytest_ant.log
timeout -k 10 300 python tools/bench_neuro.py > gpurun_out/bench_neuro.log 2>&1 && tail -1 gpurun_out/bench_neuro.log
R=$GRAFT_REPO_ROOT
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_cma -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 3 > $R/gpurun_out/prof_cma.log 2>&1 || { tail -20 $R/gpurun_out/prof_cma.log; exit 1; }
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_neuro -o run --output-format csv -- python3 $R/tools/bench_neuro.py --gens 3 > $R/gpurun_out/prof_neuro.log 2>&1 || { tail -20 $R/gpurun_out/prof_neuro.log; exit 1; }
cd $R; for d in prof_cma prof_neuro; do f=$(find gpurun_out/$d -name '*kernel_stats.csv' | head -1); echo $f; head -14 "$f" | cut -c1-200; done
