set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/s17
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/test_eigh_sbr.py tests/test_sbr_device_gpu.py -x -p no:cacheprovider > gpurun_out/s17/t.log 2>&1 || { tail -30 gpurun_out/s17/t.log | cut -c1-300; exit 1; }
tail -2 gpurun_out/s17/t.log
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > gpurun_out/s17/b20.log 2>&1 && tail -1 gpurun_out/s17/b20.log | cut -c1-250
timeout -k 10 200 python -u bench.py --steps 50 --warmup 5 > gpurun_out/s17/b50.log 2>&1 && tail -1 gpurun_out/s17/b50.log | cut -c1-250
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/s17/kt -o kt --output-format csv -- python3 $R/bench.py --steps 40 --warmup 5 --phase-steps 0 > $R/gpurun_out/s17/kt_bench.log 2>&1 || { cd $R; tail -20 gpurun_out/s17/kt_bench.log; exit 1; }
cd $R
f=$(find gpurun_out/s17/kt -name '*kernel_trace.csv' | head -1)
python tools/ktrace_gen.py $f --marker philox_h --show -2 --agg 20 > gpurun_out/s17/kt_gen.txt
grep "sbr16_block\|=== last" -A1 gpurun_out/s17/kt_gen.txt | cut -c1-160 | tail -6
rm -f $f
