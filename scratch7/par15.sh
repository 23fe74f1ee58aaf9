set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/s33
PYTHONPATH=. timeout -k 10 1100 python -u tools/parity_probe15.py gpurun_out/s33/traj.jsonl > gpurun_out/s33/log.txt 2>&1 || { tail -5 gpurun_out/s33/log.txt; exit 1; }
tail -3 gpurun_out/s33/log.txt
