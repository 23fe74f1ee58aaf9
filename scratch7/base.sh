set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/s7
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/s7/base_b20.json 2>gpurun_out/s7/base.err || { tail gpurun_out/s7/base.err; exit 1; }
tail -1 gpurun_out/s7/base_b20.json | cut -c1-400
timeout -k 10 200 python bench.py --steps 50 --warmup 5 > gpurun_out/s7/base_b50.json 2>>gpurun_out/s7/base.err || { tail gpurun_out/s7/base.err; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/s7/base_b50.json').read().strip().splitlines()[-1]);print(d['ms_per_step'],d['phases_ms_eager'],d['eigh_stats']['iters_per_gen'])"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/s7/kt -o kt --output-format csv -- python3 $R/bench.py --steps 40 --warmup 5 --phase-steps 0 > $R/gpurun_out/s7/kt_bench.log 2>&1 || { cd $R; tail -20 gpurun_out/s7/kt_bench.log; exit 1; }
cd $R
f=$(find gpurun_out/s7/kt -name '*kernel_trace.csv' | head -1)
python tools/ktrace_gen.py $f --marker philox_h --show -2 --agg 20 > gpurun_out/s7/kt_gen.txt
grep -A40 "=== last" gpurun_out/s7/kt_gen.txt | cut -c1-160
rm -f $f
