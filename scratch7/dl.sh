set -e
mkdir -p gpurun_out/dl
PYTHONPATH=. timeout -k 10 300 python -u scratch7/dl.py > gpurun_out/dl/out.txt 2>&1
PYTHONPATH=. timeout -k 10 300 python -u scratch7/dl2.py > gpurun_out/dl/out2.txt 2>&1
