set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/s23
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > gpurun_out/s23/b20.log 2>&1 && tail -1 gpurun_out/s23/b20.log | cut -c1-200
python -c "import json;d=json.loads(open('gpurun_out/s23/b20.log').read().strip().splitlines()[-1]);print(d['ms_per_step'], d['config']['hipgraph'])"
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 1 --force-dist --steps 20 --warmup 5 > gpurun_out/s23/fd.log 2>&1 || { tail -20 gpurun_out/s23/fd.log; exit 1; }
python -c "import json;d=json.loads([l for l in open('gpurun_out/s23/fd.log').read().strip().splitlines() if l.startswith('{')][-1]);print('force-dist', d['ms_per_step'], d['config']['hipgraph'], d.get('rccl_world'), d.get('dist_backend'))"
