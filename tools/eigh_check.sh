set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -m evoxmi.ops.build > gpurun_out/build.log 2>&1 || { tail -30 gpurun_out/build.log; exit 1; }
timeout -k 10 300 python -m pytest tests -x -q -m gpu -k "eigh or jacobi or cma or CMA" > gpurun_out/pytest_eigh.log 2>&1 || { tail -30 gpurun_out/pytest_eigh.log; exit 1; }
tail -2 gpurun_out/pytest_eigh.log

timeout -k 10 300 python bench.py --steps 30 --warmup 3 > gpurun_out/bench.log 2>&1 && tail -1 gpurun_out/bench.log | cut -c1-200
