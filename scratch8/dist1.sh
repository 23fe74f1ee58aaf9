set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/dist1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --steps 20 --warmup 5 --force-dist > gpurun_out/dist1/fd.log 2>&1 || { tail -20 gpurun_out/dist1/fd.log; exit 1; }
grep '"metric"' gpurun_out/dist1/fd.log | python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['ms_per_step'], d['rccl_world'], d['dist_backend'], d['config']['hipgraph'], d['eigh_stats']['capped'], d['eigh_stats']['schedule_per_gen'])"
timeout -k 10 120 python bench.py --gpus 2 --steps 2 --warmup 1 > gpurun_out/dist1/g2.log 2>&1; echo "gpus2 rc=$?"; tail -2 gpurun_out/dist1/g2.log
