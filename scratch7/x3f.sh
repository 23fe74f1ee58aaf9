set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/s9
timeout -k 10 300 python tools/xnorm_probe.py --gens 30 --solves 2 > gpurun_out/s9/xnorm.jsonl 2>gpurun_out/s9/err || { tail gpurun_out/s9/err; exit 1; }
cat gpurun_out/s9/xnorm.jsonl | cut -c1-300
timeout -k 10 300 python tools/xnorm_probe.py --gens 8 --solves 1 > gpurun_out/s9/xnorm8.jsonl 2>>gpurun_out/s9/err || { tail gpurun_out/s9/err; exit 1; }
cat gpurun_out/s9/xnorm8.jsonl | cut -c1-300
