set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/s16
PYTHONPATH=. timeout -k 10 120 python -u scratch7/rngprobe.py > gpurun_out/s16/rng.json 2>&1 || { tail gpurun_out/s16/rng.json; exit 1; }
tail -1 gpurun_out/s16/rng.json
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_gemm_blk.py tests/test_random.py -x -p no:cacheprovider > gpurun_out/s16/t.log 2>&1 || { tail -30 gpurun_out/s16/t.log; exit 1; }
tail -2 gpurun_out/s16/t.log
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/s16/kt -o kt --output-format csv -- python3 $R/bench.py --steps 40 --warmup 5 --phase-steps 0 > $R/gpurun_out/s16/kt_bench.log 2>&1 || { cd $R; tail -20 gpurun_out/s16/kt_bench.log; exit 1; }
cd $R
f=$(find gpurun_out/s16/kt -name '*kernel_trace.csv' | head -1)
python tools/ktrace_gen.py $f --marker philox_h --show -2 --agg 20 > gpurun_out/s16/kt_gen.txt
grep "philox_h" gpurun_out/s16/kt_gen.txt | cut -c1-160 | tail -3
rm -f $f
