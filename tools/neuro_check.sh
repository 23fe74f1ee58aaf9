set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -m evoxmi.ops.build > gpurun_out/build.log 2>&1 || { tail -30 gpurun_out/build.log; exit 1; }
timeout -k 10 300 python -m pytest tests -x -q -m gpu -k "ant" > gpurun_out/pytest_ant.log 2>&1 || { tail -30 gpurun_out/pytest_ant.log; exit 1; }
tail -2 gpurun_out/pytest_ant.log
timeout -k 10 300 python tools/bench_neuro.py > gpurun_out/bench_neuro.log 2>&1 && tail -1 gpurun_out/bench_neuro.log
timeout -k 10 300 python tools/bench_neuro.py --kernel-only > gpurun_out/bench_neuro_k.log 2>&1 && tail -1 gpurun_out/bench_neuro_k.log
timeout -k 10 300 python tools/bench_neuro.py --kernel-only --hidden 128 > gpurun_out/bench_neuro_k128.log 2>&1 && tail -1 gpurun_out/bench_neuro_k128.log
