set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for pop in 256 1024 2048 8192; do for cap in 50 1000; do
timeout -k 10 120 python tools/bench_neuro.py --kernel-only --pop $pop --cap $cap --wscale 0.0 >> gpurun_out/neuro_sweep.log 2>&1 || exit 1
done; done
grep kernel_only gpurun_out/neuro_sweep.log
