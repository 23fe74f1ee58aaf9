set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/dist
TR="python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1"
timeout -k 10 300 $TR --master-port 29601 bench.py --force-dist --steps 20 --warmup 3 > gpurun_out/dist/bench_graph.log 2>&1
echo "bench_graph rc=$?" >> gpurun_out/dist/rc.log
timeout -k 10 300 $TR --master-port 29602 bench.py --force-dist --no-graph --steps 20 --warmup 3 > gpurun_out/dist/bench_eager.log 2>&1
echo "bench_eager rc=$?" >> gpurun_out/dist/rc.log
timeout -k 10 300 $TR --master-port 29603 tools/bench_neuro.py --force-dist --gens 3 > gpurun_out/dist/neuro_eager.log 2>&1
echo "neuro_eager rc=$?" >> gpurun_out/dist/rc.log
timeout -k 10 300 python tools/bench_neuro.py --gens 3 --graph > gpurun_out/dist/neuro_graph1.log 2>&1
echo "neuro_graph1 rc=$?" >> gpurun_out/dist/rc.log
