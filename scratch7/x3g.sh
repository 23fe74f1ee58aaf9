set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/s10
timeout -k 10 300 python tools/xnorm_probe.py --gens 12 --from 8 > gpurun_out/s10/xnorm_warm.jsonl 2>gpurun_out/s10/err || { tail gpurun_out/s10/err; exit 1; }
cut -c1-330 gpurun_out/s10/xnorm_warm.jsonl
timeout -k 10 300 python tools/xnorm_probe.py --gens 32 --from 30 > gpurun_out/s10/xnorm_late.jsonl 2>>gpurun_out/s10/err || { tail gpurun_out/s10/err; exit 1; }
cut -c1-330 gpurun_out/s10/xnorm_late.jsonl
timeout -k 10 600 python tools/parity_probe.py --sets 3 > gpurun_out/s10/parity.jsonl 2>>gpurun_out/s10/err || { tail gpurun_out/s10/err; exit 1; }
cut -c1-600 gpurun_out/s10/parity.jsonl
