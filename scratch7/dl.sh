set -e
mkdir -p gpurun_out/dl
PYTHONPATH=. timeout -k 10 300 python -u scratch7/it.py > gpurun_out/dl/it.txt 2>&1
