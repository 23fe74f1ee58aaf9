# CEC basic-function kernel with the fused f < 1e-8 clamp: CEC tests + bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "cec or CEC or graph or bench" > gpurun_out/r3av_tests.log 2>&1 || { tail -40 gpurun_out/r3av_tests.log; exit 1; }
tail -2 gpurun_out/r3av_tests.log
for i in 1 2; do
timeout -k 10 300 python bench.py --steps 50 --warmup 3 > gpurun_out/r3av_bench50_$i.log 2>&1 || { tail -30 gpurun_out/r3av_bench50_$i.log; exit 1; }
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('50 steps', d['ms_per_step'], d['eigh_stats']['max_off_rel'])" gpurun_out/r3av_bench50_$i.log
done
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/r3av_bench20.log 2>&1 || { tail -30 gpurun_out/r3av_bench20.log; exit 1; }
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('20 steps', d['ms_per_step'])" gpurun_out/r3av_bench20.log
